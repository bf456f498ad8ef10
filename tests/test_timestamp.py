"""CPU: files.modified as chrono's DateTime<Utc> (src/index.rs:176-218, 616-619).

The writer follows chrono 0.4's to_rfc3339 (0/3/6/9 fractional digits,
"+00:00"); the reader accepts what DateTime::parse_from_rfc3339 / rusqlite's
naive fallback accept, and the mtime gate compares instants.  Parity with
rusqlite's exact writer is unpinned (its source is not vendored): these tests
pin the restatement's own properties -- ns round trips and value comparison."""
import datetime as dt
import os
from pathlib import PurePath

import pytest

from syncfast_amd.index import Index, _mtime
from syncfast_amd.timestamp import DateTimeUtc

NS = 1_000_000_000
BASE = 1_700_000_000 * NS  # 2023-11-14T22:13:20Z


@pytest.mark.parametrize("nanos,text", [
    (0, "2023-11-14T22:13:20+00:00"),
    (500_000_000, "2023-11-14T22:13:20.500+00:00"),
    (123_000_000, "2023-11-14T22:13:20.123+00:00"),
    (123_456_000, "2023-11-14T22:13:20.123456+00:00"),
    (1_000, "2023-11-14T22:13:20.000001+00:00"),
    (123_456_789, "2023-11-14T22:13:20.123456789+00:00"),
    (1, "2023-11-14T22:13:20.000000001+00:00"),
    (100, "2023-11-14T22:13:20.000000100+00:00"),
])
def test_to_sql_chrono_rfc3339_digits(nanos, text):
    t = DateTimeUtc.from_ns(BASE + nanos)
    assert t.to_sql() == text
    assert DateTimeUtc.from_sql(text) == t


def test_epoch_and_before():
    assert DateTimeUtc(0).to_sql() == "1970-01-01T00:00:00+00:00"
    t = DateTimeUtc(-1)  # one ns before the epoch
    assert t.to_sql() == "1969-12-31T23:59:59.999999999+00:00"
    assert DateTimeUtc.from_sql(t.to_sql()) == t


@pytest.mark.parametrize("text", [
    "2023-11-14T22:13:20.123456789Z",
    "2023-11-14T23:13:20.123456789+01:00",
    "2023-11-14T20:43:20.123456789-01:30",
    "2023-11-14 22:13:20.123456789+00:00",   # space separator (rusqlite rewrites it to 'T')
    "2023-11-14 22:13:20.123456789",         # naive: read as UTC
    "2023-11-14T22:13:20.1234567891234+00:00",  # > 9 digits: truncated
])
def test_from_sql_forms_are_instants(text):
    assert DateTimeUtc.from_sql(text) == DateTimeUtc(BASE + 123_456_789)


def test_from_sql_rejects_garbage():
    with pytest.raises(ValueError):
        DateTimeUtc.from_sql("yesterday")


def test_datetime_coercion():
    d = dt.datetime(2023, 11, 14, 22, 13, 20, 250000, tzinfo=dt.timezone.utc)
    assert DateTimeUtc.coerce(d) == DateTimeUtc(BASE + 250_000_000)
    assert DateTimeUtc.coerce(d).to_datetime() == d
    assert DateTimeUtc.coerce(BASE) == DateTimeUtc(BASE)


def test_gate_compares_instants_at_ns_precision():
    idx = Index.open_in_memory()
    t = DateTimeUtc(BASE + 123_456_789)
    assert idx.add_file("f", t) == (1, False)
    assert idx.db.execute("SELECT modified FROM files").fetchone()[0] == "2023-11-14T22:13:20.123456789+00:00"
    assert idx.add_file("f", DateTimeUtc(BASE + 123_456_789)) == (1, True)
    assert idx.add_file("f", DateTimeUtc(BASE + 123_456_790)) == (1, False)  # 1 ns later: modified
    assert idx.get_file("f")[1] == DateTimeUtc(BASE + 123_456_790)
    assert idx.list_files()[0][2] == DateTimeUtc(BASE + 123_456_790)


def test_gate_reads_other_writers_text_by_value():
    # a row written with a different but equivalent text (fixed 6 digits, a
    # 'Z', a space separator) is the same instant: up to date, not re-indexed
    idx = Index.open_in_memory()
    for i, text in enumerate(["2023-11-14T22:13:20.500000+00:00", "2023-11-14T22:13:20.5Z",
                              "2023-11-14 22:13:20.500"]):
        name = f"f{i}"
        idx.db.execute("INSERT INTO files(name, modified, temporary) VALUES(?, ?, 0);", (name, text))
        fid = idx.get_file(name)[0]
        assert idx.add_file(name, DateTimeUtc(BASE + 500_000_000)) == (fid, True), text
        assert idx.add_file(name, DateTimeUtc(BASE + 500_000_001)) == (fid, False), text


def test_mtime_of_open_file_keeps_nanoseconds(tmp_path):
    p = tmp_path / "x"
    p.write_bytes(b"abc")
    os.utime(p, ns=(BASE + 7, BASE + 123_456_789))
    st_ns = os.stat(p).st_mtime_ns  # the filesystem may round; the gate sees what it stores
    with open(p, "rb") as f:
        m = _mtime(f)
    assert m == DateTimeUtc(st_ns)
    idx = Index.open_in_memory()
    assert idx.add_file(PurePath("x"), m)[1] is False
    with open(p, "rb") as f:
        assert idx.add_file(PurePath("x"), _mtime(f))[1] is True
    os.utime(p, ns=(BASE, st_ns + 1000))
    with open(p, "rb") as f:
        assert idx.add_file(PurePath("x"), _mtime(f))[1] is False
