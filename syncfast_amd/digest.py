"""HashDigest -- the signature value type (/root/reference/src/lib.rs:72-145).

20 raw SHA-1 bytes (HASH_DIGEST_LEN, src/lib.rs:72) in sha1.digest().bytes()
order.  Stored in SQLite as 40 lowercase hex characters (ToSql,
src/lib.rs:78-90), parsed back with the same two error cases as FromSql
(src/lib.rs:92-136), displayed as hex (src/lib.rs:138-145).
"""
from __future__ import annotations

import re

HASH_DIGEST_LEN = 20
_HEX_PAIR = re.compile(r"\+?[0-9a-fA-F]{1,2}")


class InvalidHashDigest(ValueError):
    """FromSql failure: 'Invalid hash: wrong size' / 'Invalid hash: invalid character'."""


class HashDigest:
    __slots__ = ("_b",)

    def __init__(self, raw: bytes):
        raw = bytes(raw)
        if len(raw) != HASH_DIGEST_LEN:
            raise ValueError(f"HashDigest needs {HASH_DIGEST_LEN} bytes, got {len(raw)}")
        self._b = raw

    @property
    def bytes(self) -> bytes:
        return self._b

    def to_sql(self) -> str:
        """Lowercase hex, as write!("{:02x}") per byte (src/lib.rs:78-90)."""
        return self._b.hex()

    @classmethod
    def from_sql(cls, value) -> "HashDigest":
        """src/lib.rs:113-136: exactly 40 chars, each pair a hex byte."""
        if not isinstance(value, str):
            raise InvalidHashDigest("Invalid hash: not text")
        if len(value) != 40:
            raise InvalidHashDigest("Invalid hash: wrong size")
        out = bytearray(HASH_DIGEST_LEN)
        for i in range(HASH_DIGEST_LEN):
            pair = value[2 * i:2 * i + 2]
            # u8::from_str_radix(pair, 16): optional '+', then hex digits only
            if not _HEX_PAIR.fullmatch(pair):
                raise InvalidHashDigest("Invalid hash: invalid character")
            out[i] = int(pair, 16)
        return cls(bytes(out))

    def __str__(self) -> str:
        return self._b.hex()

    def __repr__(self) -> str:
        return f"HashDigest({self._b.hex()})"

    def __eq__(self, other) -> bool:
        return isinstance(other, HashDigest) and other._b == self._b

    def __hash__(self) -> int:
        return hash(self._b)
