"""``chrono::DateTime<Utc>`` as the index stores it (the ``files.modified`` column).

The reference takes a file's mtime as ``file.metadata()?.modified()?.into()``
(/root/reference/src/index.rs:616-619): a ``SystemTime`` converted to
``DateTime<Utc>`` with its full nanosecond precision.  rusqlite 0.16's chrono
support (``Cargo.toml:23``, ``Cargo.lock`` chrono 0.4.19) writes it with
``to_rfc3339()`` and reads it back with ``DateTime::parse_from_rfc3339`` (falling
back to a naive "YYYY-MM-DD HH:MM:SS[.f]" read as UTC); ``add_file``'s mtime
gate compares the parsed VALUES (``old_modified != modified``,
src/index.rs:183), not the text.

chrono's RFC 3339 writer (``Fixed::RFC3339`` = NaiveDate/NaiveTime ``Debug`` +
``+00:00``) prints the fraction with 0, 3, 6 or 9 digits: none when the
nanoseconds are 0, else the shortest of millis / micros / nanos that is exact.

Parity is UNPINNED: rusqlite's and chrono's sources are not vendored in
/root/reference, so the writer and reader above are restated from their
published behaviour, not checked against a reference-written index.  The
restatement is exact for what matters to the gate: the value round-trips with
nanosecond precision, and any text chrono can parse (Z or +HH:MM offsets, any
fraction length, a space separator) compares by instant.
"""
from __future__ import annotations

import datetime as _dt
import re
from dataclasses import dataclass

_EPOCH = _dt.datetime(1970, 1, 1, tzinfo=_dt.timezone.utc)
_NS = 1_000_000_000

_RFC3339 = re.compile(
    r"^(?P<date>[+-]?\d{4,}-\d{2}-\d{2})[Tt ](?P<h>\d{2}):(?P<m>\d{2}):(?P<s>\d{2})(?:\.(?P<f>\d+))?"
    r"(?P<tz>[Zz]|[+-]\d{2}:\d{2})?$")


@dataclass(frozen=True)
class DateTimeUtc:
    """A UTC instant with nanosecond precision (``ns`` since the Unix epoch)."""
    ns: int

    @classmethod
    def from_ns(cls, ns: int) -> "DateTimeUtc":
        return cls(int(ns))

    @classmethod
    def from_datetime(cls, dt: _dt.datetime) -> "DateTimeUtc":
        """An aware datetime (a naive one is taken as UTC); microsecond precision."""
        if dt.tzinfo is None:
            dt = dt.replace(tzinfo=_dt.timezone.utc)
        delta = dt - _EPOCH
        return cls((delta.days * 86400 + delta.seconds) * _NS + delta.microseconds * 1000)

    @classmethod
    def coerce(cls, v) -> "DateTimeUtc":
        if isinstance(v, DateTimeUtc):
            return v
        if isinstance(v, _dt.datetime):
            return cls.from_datetime(v)
        if isinstance(v, int):
            return cls(v)
        raise TypeError(f"cannot use {type(v).__name__} as a DateTime<Utc>")

    def to_datetime(self) -> _dt.datetime:
        """As a Python datetime (truncated to microseconds)."""
        secs, nanos = divmod(self.ns, _NS)
        return _EPOCH + _dt.timedelta(seconds=secs, microseconds=nanos // 1000)

    def to_sql(self) -> str:
        """chrono 0.4 ``to_rfc3339()``: YYYY-MM-DDTHH:MM:SS[.fff|.ffffff|.fffffffff]+00:00."""
        secs, nanos = divmod(self.ns, _NS)
        days, sod = divmod(secs, 86400)
        date = _dt.date(1970, 1, 1) + _dt.timedelta(days=days)
        y = date.year
        ytxt = f"{y:04d}" if 0 <= y <= 9999 else f"{y:+05d}"
        h, rem = divmod(sod, 3600)
        m, s = divmod(rem, 60)
        if nanos == 0:
            frac = ""
        elif nanos % 1_000_000 == 0:
            frac = f".{nanos // 1_000_000:03d}"
        elif nanos % 1000 == 0:
            frac = f".{nanos // 1000:06d}"
        else:
            frac = f".{nanos:09d}"
        return f"{ytxt}-{date.month:02d}-{date.day:02d}T{h:02d}:{m:02d}:{s:02d}{frac}+00:00"

    @classmethod
    def from_sql(cls, text) -> "DateTimeUtc":
        """rusqlite's ``FromSql for DateTime<Utc>``: RFC 3339 (a space may
        stand for the 'T'), else a naive date-time read as UTC.  Fractions
        beyond 9 digits are truncated, as chrono's parser does."""
        if isinstance(text, bytes):
            text = text.decode()
        mt = _RFC3339.match(str(text).strip())
        if not mt:
            raise ValueError(f"not an RFC 3339 / naive date-time: {text!r}")
        y, mo, d = (int(x) for x in re.match(r"^([+-]?\d+)-(\d+)-(\d+)$", mt["date"]).groups())
        days = (_dt.date(y, mo, d) - _dt.date(1970, 1, 1)).days
        frac = (mt["f"] or "")[:9].ljust(9, "0")
        ns = ((days * 86400 + int(mt["h"]) * 3600 + int(mt["m"]) * 60 + int(mt["s"])) * _NS + int(frac))
        tz = mt["tz"]
        if tz and tz not in ("Z", "z"):
            sign = 1 if tz[0] == "+" else -1
            hh, mm = int(tz[1:3]), int(tz[4:6])
            ns -= sign * (hh * 3600 + mm * 60) * _NS
        return cls(ns)

    def __str__(self) -> str:
        return self.to_sql()
