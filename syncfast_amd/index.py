"""Index -- syncfast's library index API with the signatures computed on MI355X.

Mirrors ``pub struct Index`` (/root/reference/src/index.rs:43-736): the same
SQLite schema (src/index.rs:12-38), the same methods and row semantics, so
callers written against the reference (the CLI ``index`` command,
src/main.rs:111-124, and the sync endpoints, src/sync/fs.rs:53-58, 239-248,
463) see identical data.  What changes is the hot path inside
``index_file`` (src/index.rs:610-659): instead of a per-byte CPU loop and one
SQL INSERT per block, the file's bytes go through the C-ABI to the gfx950
SHA-1 kernel and the rows are inserted in one batch.

Chunking -- an explicit choice, there is no default.  The reference cuts
blocks with the third-party cdchunking 0.2.1 ZPAQ chunker (src/index.rs:
622-625), whose recurrence is not available here (CDC parity
unpinned).  ``index_file`` / ``index_path`` therefore need the chunker the
caller chose when opening the index:
  * ``BoundaryChunker(fn)`` -- the reference's mode: the boundary function is
    the host chunker (in a Rust drop-in, the cdchunking crate itself), so the
    blocks are the reference's by construction; every block's SHA-1 and the
    ``blocks_hash`` come from the GPU.  ``stream=True`` hands ``fn`` the open
    file (as ``chunker.stream(file)`` reads it) and the library re-reads the
    same open file by windows (sf_index_fd_blocks), so no file is held whole;
  * ``FixedChunker(block_size)`` -- fixed tiling, the BASELINE configs' mode.
    NOT the reference's default blocks: an index built this way only works
    with peers that use the same mode and read a block as its row's
    ``(offset, size)`` bytes (``read_block`` below), never by re-chunking
    from the offset as the reference's ``read_block`` does
    (src/sync/fs.rs:26-40).
The per-block SHA-1, the rows, ``blocks_hash`` and every query are
bit-identical to the reference for the same boundaries.  An ``Index`` opened
without a chunker serves every query but refuses to index.

Timestamps.  ``files.modified`` is a ``DateTime<Utc>`` (``timestamp.DateTimeUtc``):
taken from the open file's metadata with nanosecond precision
(src/index.rs:616-619), written as chrono's RFC 3339 text and compared as a
parsed value in the mtime gate (src/index.rs:183) -- see timestamp.py (parity
with rusqlite's exact writer is unpinned).

Walk order.  ``index_path`` visits directory entries in ``os.listdir`` order,
which is readdir(3) order -- the order Rust's ``read_dir`` yields
(src/index.rs:698) -- so ``file_id``s are assigned as the reference would on
the same filesystem.

Quirks kept on purpose: ``index_file`` leaves ``files.size`` NULL (the
reference never sets it there, so ``list_files`` reports 0, src/index.rs:
376-377); ``compute_blocks_hash`` hashes the digests in the order SQLite
returns them for ``WHERE file_id = ?`` with no ORDER BY (src/index.rs:663-
669), which is insertion (= offset) order.
"""
from __future__ import annotations

import ctypes
import logging
import os
import sqlite3
import stat
from pathlib import Path, PurePath
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

from . import host
from ._lib import SF_EAGAIN, SfError, same_stamp
from .digest import HashDigest
from .timestamp import DateTimeUtc

log = logging.getLogger("syncfast_amd.index")

# index_file: times a file that keeps changing while it is indexed
# (SF_EAGAIN from the descriptor routes) is opened and indexed again.
CHANGED_RETRIES = 3
# Index.index_path with a NativeChunker: a file this large is cut on the
# chunker's threads and hashed from one read (sf_index_fd_cut), not cut on one
# pool thread among the batch's files (configs[0]'s folder is one 64 MiB file).
LARGE_FILE_BYTES = 64 << 20

SCHEMA = """
    CREATE TABLE files(
        file_id INTEGER NOT NULL PRIMARY KEY,
        name VARCHAR(512) NOT NULL,
        modified DATETIME NOT NULL,
        size INTEGER NULL,
        blocks_hash VARCHAR(40) NULL,
        temporary BOOLEAN NOT NULL
    );
    CREATE INDEX idx_files_name ON files(name);

    CREATE TABLE blocks(
        file_id INTEGER NOT NULL,
        hash VARCHAR(40) NOT NULL,
        offset INTEGER NOT NULL,
        size INTEGER NOT NULL,
        present BOOLEAN NOT NULL,
        PRIMARY KEY(file_id, offset)
    );
    CREATE INDEX idx_blocks_file_id ON blocks(file_id);
    CREATE INDEX idx_blocks_hash ON blocks(hash);
    CREATE INDEX idx_blocks_offset ON blocks(file_id, offset);
    CREATE INDEX idx_blocks_present ON blocks(file_id, present);

    PRAGMA application_id=0x51367457;
    PRAGMA user_version=0x00000000;
"""

INDEX_FILE_NAME = ".syncfast.idx"  # src/index.rs:699, src/main.rs:117
TEMP_PREFIX = ".syncfast_tmp_"     # src/lib.rs:152


class SyncfastError(Exception):
    """Error (src/lib.rs:24-31): Io / Sqlite / BadFilenameEncoding."""


def temp_name(name) -> PurePath:
    """src/lib.rs:147-158: dir/file -> dir/.syncfast_tmp_file."""
    p = PurePath(name)
    if not p.name:
        raise SyncfastError("Invalid path")
    return p.with_name(TEMP_PREFIX + p.name)


def untemp_name(name) -> PurePath:
    """src/lib.rs:160-174."""
    p = PurePath(name)
    if not p.name.startswith(TEMP_PREFIX):
        raise SyncfastError("Not a temporary path")
    return p.with_name(p.name[len(TEMP_PREFIX):])


def _name_str(name) -> str:
    s = str(PurePath(name)) if str(name) != "" else ""
    try:
        s.encode("utf-8")
    except UnicodeEncodeError:
        raise SyncfastError("BadFilenameEncoding") from None
    return s


def _mtime(f) -> DateTimeUtc:
    """``file.metadata()?.modified()?.into()`` (src/index.rs:616-619): the open
    file's mtime, to the nanosecond."""
    return DateTimeUtc.from_ns(os.fstat(f.fileno()).st_mtime_ns)


def _stamp_moved(fd: int, stamp) -> bool:
    """Has the file open on fd changed since `stamp` (host.file_stamp)?"""
    return not same_stamp(host.file_stamp(fd), stamp)


def _now() -> DateTimeUtc:
    """``chrono::Utc::now()`` (src/index.rs:265)."""
    import time
    return DateTimeUtc.from_ns(time.time_ns())


# ----------------------------------------------------------------- chunkers

def _seekable(f) -> bool:
    """A regular file: the native routes map or pread it.  Anything else
    File::open accepts (a FIFO, a character device) is read sequentially from
    the open descriptor (sf_index_fd): a second open of a FIFO would wait for
    another writer."""
    return stat.S_ISREG(os.fstat(f.fileno()).st_mode)


class FixedChunker:
    """Blocks of `block_size` bytes (last one shorter); no empty blocks.

    Not the reference's blocks (those are content-defined, src/index.rs:
    622-625): use it only where every peer indexes the same way and reads a
    block by its row's (offset, size) -- see ``read_block``."""

    def __init__(self, block_size: int):
        if not 0 < block_size <= (32 << 20):
            raise ValueError("block_size must be in (0, 32 MiB]")
        self.block_size = block_size


class BoundaryChunker:
    """Blocks from a host chunker -- the reference's mode (src/index.rs:
    622-625).  fn(data: bytes) -> list of block sizes (positive, summing to
    len(data)); with ``stream=True``, fn(file) reads an open binary file to
    its end (as ``chunker.stream(file)`` does, src/index.rs:625) and returns
    the sizes, and the file is re-read by windows on the library side
    (sf_index_fd_blocks) instead of being held whole.  The signatures are
    computed by the GPU kernel (explicit-block-list entry points)."""

    def __init__(self, fn: Callable, stream: bool = False):
        self.fn = fn
        self.stream = stream


class _ChunkerOps(ctypes.Structure):
    """sf_chunker_ops (include/syncfast_amd.h)."""
    _fields_ = [("create", ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p)),
                ("next", ctypes.CFUNCTYPE(ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)),
                ("destroy", ctypes.CFUNCTYPE(None, ctypes.c_void_p)),
                ("ctx", ctypes.c_void_p)]


class NativeChunker(BoundaryChunker):
    """The reference's mode with a native chunker: ``ops`` is the address of
    an sf_chunker_ops (create / next / destroy in C: cdchunking's ZPAQ on the
    Rust side; examples/zpaq_standin_ops.c here).  The
    library runs it itself: Index.index_file cuts and hashes a file in one
    call on ``threads`` threads, the file read once (sf_index_fd_cut, the
    one-stream boundaries whatever the thread count); Index.index_path cuts
    the files on its pool (sf_cut_fd, one thread per file) and hashes them
    as batches (sf_index_fds_blocks)."""

    def __init__(self, ops: int, threads: int = 0):
        super().__init__(self._sizes, stream=True)
        self.ops = int(ops)
        self.threads = threads

    def _sizes(self, f) -> List[int]:
        if hasattr(f, "fileno"):
            try:
                fd = f.fileno()
            except (OSError, ValueError):  # io.BytesIO: the bytes of one read
                fd = None
            if fd is not None:
                return host.cut_fd(fd, self.ops, 1)[1].tolist()
        return self._cut_bytes(f.read())

    def _cut_bytes(self, raw: bytes) -> List[int]:
        """The chunker over bytes in memory, driven from here through its
        three functions (the one-pass fallback of index_file)."""
        ops = _ChunkerOps.from_address(self.ops)
        ch = ops.create(ops.ctx)
        if not ch:
            raise MemoryError("chunker create failed")
        try:
            buf = ctypes.create_string_buffer(raw, len(raw)) if raw else None
            base = ctypes.addressof(buf) if buf is not None else 0
            sizes, start, pos = [], 0, 0
            while pos < len(raw):
                k = ops.next(ch, base + pos, len(raw) - pos)
                if k == 0:
                    break
                pos += k
                sizes.append(pos - start)
                start = pos
            if start < len(raw):
                sizes.append(len(raw) - start)
            return sizes
        finally:
            ops.destroy(ch)


def _sizes_ok(sizes, n: int) -> List[int]:
    sizes = [int(x) for x in sizes]
    if any(x <= 0 for x in sizes) or sum(sizes) != n:
        raise ValueError("boundary function must return positive sizes covering the data")
    return sizes


def _offsets(sizes) -> np.ndarray:
    offs = np.zeros(len(sizes), np.uint64)
    if len(sizes) > 1:
        offs[1:] = np.cumsum(np.asarray(sizes, np.uint64), dtype=np.uint64)[:-1]
    return offs


def read_block(path, offset: int, size: int) -> bytes:
    """The bytes of one block row: `size` bytes at `offset`.

    The sync code's reader (src/sync/fs.rs:26-40) instead re-runs a fresh
    ZPAQ chunker from `offset` and returns the first chunk it cuts; for rows
    of the reference's content-defined blocks that is the same bytes (a
    chunker's state resets at every boundary), for any other
    tiling it is not.  A drop-in that indexes with fixed tiling must replace
    read_block with this ("Fixed tiling"); it is correct for
    both modes."""
    with open(path, "rb") as f:
        f.seek(offset)
        b = f.read(size)
    if len(b) != size:
        raise SyncfastError("No such chunk in file")
    return b


Chunker = object  # FixedChunker | BoundaryChunker


def signatures_of_bytes(data, chunker) -> List[Tuple[int, int, bytes]]:
    """(offset, size, digest) rows of one file's bytes, computed on the GPU."""
    if isinstance(chunker, FixedChunker):
        return host.rows_to_tuples(host.index_buffer(data, chunker.block_size))
    if isinstance(chunker, BoundaryChunker):
        # the boundaries come from the host-side chunker, as the reference's
        # do (src/index.rs:622-625); every block's SHA-1 is computed on the
        # device through the host-memory C-ABI entry (sf_index_buffer_blocks)
        raw = bytes(data)
        import io
        sizes = _sizes_ok(chunker.fn(io.BytesIO(raw)) if chunker.stream else chunker.fn(raw), len(raw))
        if not sizes:
            return []
        rows, _ = host.index_buffer_blocks(raw, _offsets(sizes), np.asarray(sizes, np.uint32))
        return host.rows_to_tuples(rows)
    raise TypeError("unknown chunker")


# -------------------------------------------------------------------- Index

class Index:
    """Index of files and blocks (src/index.rs:43-47)."""

    def __init__(self, db: sqlite3.Connection, chunker=None):
        self.db = db
        self.in_transaction = False
        self.chunker = chunker  # None: queries only; index_file / index_path refuse

    def _need_chunker(self):
        if self.chunker is None:
            raise SyncfastError(
                "this Index was opened without a chunker: pass chunker=BoundaryChunker(fn) for the reference's "
                "content-defined blocks (fn = the host chunker, e.g. cdchunking's ZPAQ 13 / 32 KiB, "
                "src/index.rs:622-625) or chunker=FixedChunker(block_size) for fixed tiling (not the "
                "reference's blocks: peers must index the same way and read blocks by (offset, size))")
        if not isinstance(self.chunker, (FixedChunker, BoundaryChunker)):
            raise TypeError("unknown chunker")

    # -- open / transactions (src/index.rs:51-74, 729-735)
    @classmethod
    def open(cls, filename, chunker=None) -> "Index":
        exists = os.path.exists(filename)
        db = sqlite3.connect(str(filename), isolation_level=None)
        if not exists:
            log.warning("Database doesn't exist, creating tables...")
            db.executescript(SCHEMA)
        return cls(db, chunker)

    @classmethod
    def open_in_memory(cls, chunker=None) -> "Index":
        db = sqlite3.connect(":memory:", isolation_level=None)
        db.executescript(SCHEMA)
        return cls(db, chunker)

    def begin(self) -> None:
        if not self.in_transaction:
            self.db.execute("BEGIN IMMEDIATE;")
            self.in_transaction = True

    def commit(self) -> None:
        if self.in_transaction:
            self.db.execute("COMMIT")
            self.in_transaction = False

    # -- queries (src/index.rs:77-384, 453-607)
    def get_block(self, hash: HashDigest) -> Optional[Tuple[PurePath, int, int]]:
        row = self.db.execute(
            "SELECT files.name, blocks.offset, blocks.size FROM blocks "
            "INNER JOIN files ON blocks.file_id = files.file_id "
            "WHERE blocks.hash = ? AND blocks.present = 1;", (hash.to_sql(),)).fetchone()
        return (PurePath(row[0]), int(row[1]), int(row[2])) if row else None

    def get_blocks(self, hashes: Sequence[HashDigest], device=None) -> List[Optional[Tuple[PurePath, int, int]]]:
        """get_block for a whole list of hashes -- a FILE_BLOCK run as the
        destination receives it (src/sync/fs.rs:461-476) -- answered by one
        device lookup (syncfast_amd.device.BlockSet, sf_block_set_*): the
        index's rows in rowid order go to the GPU as a hash table, and each
        hash gets the row get_block would return (present, joined to a file,
        first in rowid order), or None."""
        import torch

        from .device import BlockSet
        rows = self.db.execute(
            "SELECT blocks.hash, blocks.present = 1 AND files.file_id IS NOT NULL, files.name, blocks.offset, "
            "blocks.size FROM blocks LEFT JOIN files ON blocks.file_id = files.file_id "
            "ORDER BY blocks.rowid;").fetchall()
        if not hashes:
            return []
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        table = np.frombuffer(bytes.fromhex("".join(r[0] for r in rows)), np.uint8).reshape(-1, 20)
        present = np.fromiter((bool(r[1]) for r in rows), bool, len(rows))
        q = np.frombuffer(b"".join(h.bytes for h in hashes), np.uint8).reshape(-1, 20)
        t = torch.from_numpy(table.copy()).to(dev)
        with BlockSet(t, torch.from_numpy(present).to(dev)) as bset:
            found = bset.lookup(torch.from_numpy(q.copy()).to(dev)).cpu().numpy()
        return [None if r < 0 else (PurePath(rows[r][2]), int(rows[r][3]), int(rows[r][4])) for r in found]

    def get_file(self, name) -> Optional[Tuple[int, DateTimeUtc, Optional[HashDigest]]]:
        row = self.db.execute(
            "SELECT file_id, modified, blocks_hash FROM files WHERE name = ? AND temporary = 0;",
            (_name_str(name),)).fetchone()
        if not row:
            return None
        return (int(row[0]), DateTimeUtc.from_sql(row[1]),
                HashDigest.from_sql(row[2]) if row[2] is not None else None)

    def get_temp_file(self, name) -> Optional[Tuple[int, DateTimeUtc]]:
        row = self.db.execute("SELECT file_id, modified FROM files WHERE name = ? AND temporary = 1;",
                              (_name_str(temp_name(name)),)).fetchone()
        return (int(row[0]), DateTimeUtc.from_sql(row[1])) if row else None

    def get_file_name(self, file_id: int) -> Optional[PurePath]:
        row = self.db.execute("SELECT name FROM files WHERE file_id = ?;", (file_id,)).fetchone()
        return PurePath(row[0]) if row else None

    def list_files(self):
        rows = self.db.execute(
            "SELECT file_id, name, modified, size, blocks_hash FROM files WHERE temporary = 0;").fetchall()
        return [(int(r[0]), PurePath(r[1]), DateTimeUtc.from_sql(r[2]), int(r[3] or 0),
                 HashDigest.from_sql(r[4]) if r[4] is not None else None) for r in rows]

    def list_file_blocks(self, file_id: int) -> List[Tuple[HashDigest, int, int]]:
        rows = self.db.execute("SELECT hash, offset, size FROM blocks WHERE file_id = ?;", (file_id,)).fetchall()
        return [(HashDigest.from_sql(r[0]), int(r[1]), int(r[2])) for r in rows]

    def list_temp_files(self) -> List[PurePath]:
        return [PurePath(r[0]) for r in self.db.execute("SELECT name FROM files WHERE temporary = 1;")]

    def check_temp_files(self):
        rows = self.db.execute(
            "SELECT file_id, name, EXISTS (SELECT hash FROM blocks WHERE blocks.file_id = files.file_id "
            "AND present = 0) AS missing FROM files WHERE temporary = 1;").fetchall()
        return [(int(r[0]), PurePath(r[1]), bool(r[2])) for r in rows]

    def list_missing_blocks(self) -> List[HashDigest]:
        return [HashDigest.from_sql(r[0]) for r in self.db.execute("SELECT hash FROM blocks WHERE present = 0;")]

    def list_block_locations(self, hash: HashDigest):
        rows = self.db.execute(
            "SELECT files.file_id, files.name, blocks.offset, blocks.size FROM blocks "
            "INNER JOIN files ON files.file_id = blocks.file_id WHERE hash = ?;", (hash.to_sql(),)).fetchall()
        return [(int(r[0]), PurePath(r[1]), int(r[2]), int(r[3])) for r in rows]

    # -- mutations (src/index.rs:176-408, 433-451, 591-607)
    def add_file(self, name, modified) -> Tuple[int, bool]:
        """(file_id, up_to_date): the mtime gate of src/index.rs:176-218.
        ``modified``: DateTimeUtc, an aware datetime, or ns since the epoch;
        compared with the stored value as an instant (src/index.rs:183)."""
        self.begin()
        m = DateTimeUtc.coerce(modified)
        ts = m.to_sql()
        cur = self.get_file(name)
        if cur is not None:
            file_id, old_modified, _ = cur
            if old_modified != m:
                log.info("Resetting file %s, modified", name)
                self.db.execute("DELETE FROM blocks WHERE file_id = ?;", (file_id,))
                self.db.execute("UPDATE files SET modified = ?, size = NULL, blocks_hash = NULL, temporary = 0 "
                                "WHERE file_id = ?;", (ts, file_id))
                return file_id, False
            return file_id, True
        log.info("Inserting new file %s", name)
        c = self.db.execute("INSERT INTO files(name, modified, temporary) VALUES(?, ?, 0);", (_name_str(name), ts))
        return int(c.lastrowid), False

    def add_file_overwrite(self, name, modified) -> int:
        self.begin()
        ts = DateTimeUtc.coerce(modified).to_sql()
        cur = self.get_file(name)
        if cur is not None:
            file_id = cur[0]
            self.db.execute("DELETE FROM blocks WHERE file_id = ?;", (file_id,))
            self.db.execute("UPDATE files SET modified = ?, size = NULL, blocks_hash = NULL, temporary = 0 "
                            "WHERE file_id = ?;", (ts, file_id))
            return file_id
        c = self.db.execute("INSERT INTO files(name, modified, temporary) VALUES(?, ?, 0);", (_name_str(name), ts))
        return int(c.lastrowid)

    def add_temp_file(self, name) -> int:
        self.begin()
        ts = _now().to_sql()
        tname = _name_str(temp_name(name))
        row = self.db.execute("SELECT file_id FROM files WHERE name = ? AND temporary = 0;", (tname,)).fetchone()
        if row is not None:
            file_id = int(row[0])
            self.db.execute("DELETE FROM blocks WHERE file_id = ?;", (file_id,))
            self.db.execute("UPDATE files SET modified = ?, size = NULL, blocks_hash = NULL, temporary = 1 "
                            "WHERE file_id = ?;", (ts, file_id))
            return file_id
        c = self.db.execute("INSERT INTO files(name, modified, temporary) VALUES(?, ?, 1);", (tname, ts))
        return int(c.lastrowid)

    def remove_file(self, file_id: int) -> None:
        self.begin()
        self.db.execute("DELETE FROM blocks WHERE file_id = ?;", (file_id,))
        self.db.execute("DELETE FROM files WHERE file_id = ?;", (file_id,))

    def move_temp_file_into_place(self, file_id: int, destination) -> None:
        self.begin()
        dst = _name_str(destination)
        self.db.execute("DELETE FROM blocks WHERE file_id = (SELECT file_id FROM files WHERE name = ?);", (dst,))
        self.db.execute("DELETE FROM files WHERE name = ?;", (dst,))
        self.db.execute("UPDATE files SET name = ?, temporary = 0 WHERE file_id = ?;", (dst, file_id))

    def add_block(self, hash: HashDigest, file_id: int, offset: int, size: int) -> None:
        """One row, present = 1 (src/index.rs:387-408)."""
        self.begin()
        self.db.execute("INSERT INTO blocks(hash, file_id, offset, size, present) VALUES(?, ?, ?, ?, 1);",
                        (hash.to_sql(), file_id, offset, size))

    def add_blocks(self, file_id: int, rows: Sequence[Tuple[int, int, bytes]]) -> None:
        """add_block for a whole signature table in one executemany (the
        reference issues one un-prepared INSERT per block)."""
        self.begin()
        self.db.executemany("INSERT INTO blocks(hash, file_id, offset, size, present) VALUES(?, ?, ?, ?, 1);",
                            ((d.hex(), file_id, o, s) for o, s, d in rows))

    def add_missing_block(self, hash: HashDigest, file_id: int, offset: int, size: int) -> None:
        self.begin()
        self.db.execute("INSERT INTO blocks(hash, file_id, offset, size, present) VALUES(?, ?, ?, ?, 0);",
                        (hash.to_sql(), file_id, offset, size))

    def mark_block_present(self, file_id: int, hash: HashDigest, offset: int) -> None:
        self.begin()
        self.db.execute("UPDATE blocks SET present = 1 WHERE file_id = ? AND hash = ? AND offset = ?;",
                        (file_id, hash.to_sql(), offset))

    def set_file_size_and_compute_blocks_hash(self, file_id: int, size: int) -> None:
        self.begin()
        bh = self.compute_blocks_hash(file_id)
        self.db.execute("UPDATE files SET size = ?, blocks_hash = ? WHERE file_id = ?;", (size, bh.to_sql(), file_id))

    def compute_blocks_hash(self, file_id: int) -> HashDigest:
        """src/index.rs:661-682: SHA-1 over the raw digests, SELECT order."""
        rows = self.db.execute("SELECT hash FROM blocks WHERE file_id = ?;", (file_id,)).fetchall()
        raw = b"".join(HashDigest.from_sql(r[0]).bytes for r in rows)
        return HashDigest(host.blocks_hash(raw))

    # -- the hot path (src/index.rs:610-659)
    def index_file(self, path, name) -> None:
        """Cut a file into blocks and add them to the index.

        Native routes return the rows and the blocks_hash together: SHA-1 over
        the digests in offset order, which is the order the rows are inserted
        in and so the order compute_blocks_hash's SELECT reads them back in
        (src/index.rs:661-682) -- the same value without re-reading the rows.
        Like the reference (src/index.rs:615-625), ONE open of the file gives
        the mtime, the boundaries and the bytes: BoundaryChunker(stream=True)
        on a regular file streams the open file and the library re-reads that
        same descriptor by windows (sf_index_fd_blocks); FixedChunker:
        sf_index_fd_fixed on it (sf_index_fd for a FIFO); a BoundaryChunker
        over bytes: the file's bytes and the list go to
        sf_index_buffer_blocks.  The descriptor routes compare the file's
        stamp (fstat, taken before the chunker read it) when they start and
        after their last read: a file written while it is indexed is indexed
        again from a new open, never stored as rows that mix two versions of
        it.  A file that keeps changing (a log being appended to) is, after
        CHANGED_RETRIES attempts, indexed in ONE pass as the reference does
        (src/index.rs:615-647): its bytes are read once from one open, the
        chunker cuts those bytes and the same bytes are hashed
        (sf_index_buffer_blocks / sf_index_buffer), so the rows describe the
        bytes read whatever the writer does meanwhile.  (Stamps are only as
        fine as the filesystem's clock tick: a same-size write within the
        tick of the stamp is not seen, include/syncfast_amd.h.)"""
        self._need_chunker()
        for attempt in range(CHANGED_RETRIES):
            try:
                self._index_file_once(path, name, force=attempt > 0)
                return
            except SfError as e:
                if e.code != SF_EAGAIN:
                    raise
                log.info("File %s changed while it was indexed, indexing it again", path)
        log.info("File %s keeps changing: indexing the bytes of one read", path)
        self._index_file_once(path, name, force=True, one_pass=True)

    def _index_file_once(self, path, name, force: bool, one_pass: bool = False, opened=None) -> None:
        """One attempt of index_file; `opened`: the file already open (a FIFO
        met by the walk is indexed from that open: a second open would wait
        for another writer, and the first's data would be lost)."""
        ch = self.chunker
        native = None  # (rows, blocks_hash) from a native route
        with (open(path, "rb") if opened is None else opened) as f:  # File::open first: same error on a missing file
            seekable = _seekable(f)
            stamp = host.file_stamp(f.fileno()) if seekable and not one_pass and \
                (isinstance(ch, FixedChunker) or ch.stream) else None
            mtime = DateTimeUtc.from_ns(stamp.mtime_sec * 10**9 + stamp.mtime_nsec) if stamp else _mtime(f)
            file_id, up_to_date = self.add_file(name, mtime)
            if up_to_date:
                if not force:
                    return
                # a retry after SF_EAGAIN whose mtime did not move (the writer
                # restored it, or only the ctime changed): index it anyway
                self.db.execute("DELETE FROM blocks WHERE file_id = ?;", (file_id,))
            if isinstance(ch, FixedChunker):
                if one_pass:  # the bytes of one read, hashed from host memory
                    raw = f.read()
                    rows_np = host.index_buffer(raw, ch.block_size)
                    native = (rows_np, host.blocks_hash(np.ascontiguousarray(rows_np["sha1"])))
                elif seekable:
                    native = host.index_fd_fixed(f.fileno(), ch.block_size, stamp)
                else:  # a FIFO: read sequentially from this open, as File::open + read do
                    native = host.index_fd(f.fileno(), ch.block_size)
            elif isinstance(ch, NativeChunker) and seekable and not one_pass:
                native = host.index_fd_cut(f.fileno(), ch.ops, ch.threads, stamp)  # cut + hash, one read
            elif ch.stream and seekable and not one_pass:
                sizes = [int(x) for x in ch.fn(f)]
                if sum(sizes) != stamp.size and _stamp_moved(f.fileno(), stamp):
                    raise SfError(SF_EAGAIN, f"index_file({os.fsdecode(path)})")  # written while chunked
                sizes = _sizes_ok(sizes, stamp.size)
                native = host.index_fd_blocks(f.fileno(), _offsets(sizes), np.asarray(sizes, np.uint32), stamp)
            else:
                rows = signatures_of_bytes(f.read(), ch)
        if native is not None:
            rows_np, bh = native
            self._insert_rows(file_id, rows_np)
            self.db.execute("UPDATE files SET blocks_hash = ? WHERE file_id = ?;", (bh.hex(), file_id))
            return
        if log.isEnabledFor(logging.DEBUG):
            for o, sz, d in rows:
                log.debug("Adding block, offset=%d, size=%d, sha1=%s", o, sz, d.hex())
        self.add_blocks(file_id, rows)
        bh = self.compute_blocks_hash(file_id)
        self.db.execute("UPDATE files SET blocks_hash = ? WHERE file_id = ?;", (bh.to_sql(), file_id))

    def _insert_rows(self, file_id: int, rows, a: int = 0, b: Optional[int] = None) -> None:
        """add_block for rows[a:b] of a native signature table: the hash column
        hex-encoded once (HashDigest ToSql, src/lib.rs:78-90), one executemany."""
        self.begin()
        b = rows.shape[0] if b is None else b
        hx = rows["sha1"][a:b].tobytes().hex()
        offs, sizes = rows["offset"][a:b].tolist(), rows["size"][a:b].tolist()
        if log.isEnabledFor(logging.DEBUG):
            for i in range(b - a):
                log.debug("Adding block, offset=%d, size=%d, sha1=%s", offs[i], sizes[i], hx[40 * i:40 * i + 40])
        self.db.executemany("INSERT INTO blocks(hash, file_id, offset, size, present) VALUES(?, ?, ?, ?, 1);",
                            ((hx[40 * i:40 * i + 40], file_id, offs[i], sizes[i]) for i in range(b - a)))

    def index_path(self, path, batch_bytes: int = 256 << 20, chunk_threads: int = 0,
                   large_file_bytes: int = LARGE_FILE_BYTES) -> None:
        """Index files and directories recursively (src/index.rs:685-715).

        Same walk, names and mtime gate as the reference.  With a
        FixedChunker, every file that needs (re)indexing goes through ONE
        native pipeline (sf_index_files) in stages of `batch_bytes`: pinned
        host buffers filled by a pread thread pool, one H2D copy and one
        device launch per stage (blocks + every file's blocks_hash), reading
        overlapped with the device.  With BoundaryChunker(stream=True) -- the
        reference's default mode -- the chunker cuts the files on a pool of
        `chunk_threads` threads (0: one per core, at most 16; a chunker is
        per-file state, so files cut independently), and every batch of about
        `batch_bytes` of cut files goes through ONE native pipeline
        (sf_index_fds_blocks: the open descriptors re-read by windows into
        packed pinned stages, one sort + one explicit-list launch per stage)
        while the pool cuts the next batch.  A NativeChunker's files of at
        least `large_file_bytes` (64 MiB: configs[0]'s one file) are instead
        cut on `chunk_threads` threads each and hashed from one read
        (sf_index_fd_cut, Index.index_file's route), in their walk position:
        one large file alone would otherwise be cut on a single thread.
        batch_bytes=0 indexes file by file."""
        self._need_chunker()
        todo: List[Tuple[Path, PurePath]] = []
        self._index_path_rec(Path(path), PurePath(""), todo)
        if not todo:
            return
        if batch_bytes <= 0:
            for p, rel in todo:
                self.index_file(p, rel)
            return
        if isinstance(self.chunker, BoundaryChunker):
            if self.chunker.stream:
                self._index_batched_fds(todo, batch_bytes, chunk_threads, large_file_bytes)
            else:
                self._index_batched_boundaries(todo, batch_bytes)
            return
        self._index_batched(todo, batch_bytes)

    def _index_path_rec(self, root: Path, rel: PurePath, todo) -> None:
        p = root / rel
        if p.is_dir():
            log.info("Indexing directory %s (%s)", rel, p)
            for entry in os.listdir(p):  # readdir order, as read_dir (src/index.rs:698)
                if entry == INDEX_FILE_NAME:
                    continue
                self._index_path_rec(root, rel / entry, todo)
        else:
            if rel.parts[:1] == (".",):
                rel = PurePath(*rel.parts[1:])
            # index_path on a file: the reference's rel is Path::new(""), whose
            # name is the empty string (PurePath("") would print as ".")
            name = "" if rel == PurePath("") else rel
            log.info("Indexing file %s (%s)", rel, p)
            todo.append((p, name))

    def _index_batched(self, todo, batch_bytes: int) -> None:
        """Every file needing (re)indexing through ONE native pipeline
        (sf_index_files): pread thread pool into pinned stages of
        `batch_bytes`, H2D + device blocks/blocks_hash per stage, overlapped
        with the reading of the next stage."""
        bs = self.chunker.block_size
        pending = []  # (file_id, path) needing signatures
        for p, rel in todo:
            with open(p, "rb") as f:  # same error as File::open on a vanished file
                file_id, up_to_date = self.add_file(rel, _mtime(f))
                if not up_to_date and not _seekable(f):
                    # a FIFO in the tree: read it from this open (a second
                    # open would wait for another writer); rows like index_file
                    rows_np, bh = host.index_fd(f.fileno(), bs)
                    self._insert_rows(file_id, rows_np)
                    self.db.execute("UPDATE files SET blocks_hash = ? WHERE file_id = ?;", (bh.hex(), file_id))
                    continue
            if not up_to_date:
                pending.append((file_id, p))
        if not pending:
            return
        rows, first, fh = host.index_files([p for _f, p in pending], bs, stage_bytes=batch_bytes)
        fhx = fh.tobytes().hex()
        for k, (file_id, _p) in enumerate(pending):
            self._insert_rows(file_id, rows, int(first[k]), int(first[k + 1]))
            self.db.execute("UPDATE files SET blocks_hash = ? WHERE file_id = ?;", (fhx[40 * k:40 * k + 40], file_id))

    def _index_batched_fds(self, todo, batch_bytes: int, chunk_threads: int,
                           large_file_bytes: int = LARGE_FILE_BYTES) -> None:
        """The default (content-defined) mode over many files, the files cut
        in parallel and hashed as ONE pipeline per batch.

        Each file is opened once and stamped (sf_file_stamp_fd: its mtime is
        the one stored, the mtime gate runs in walk order, so file_ids are the
        reference's); the chunker streams the open file on a pool thread; a
        batch of about `batch_bytes` of cut files (and at most a quarter of
        the descriptor limit) goes to sf_index_fds_blocks on those same
        descriptors while the pool cuts the next batch.  A file written while
        it was cut or read (SF_EAGAIN for it alone) is indexed again through
        index_file, in its place, so rows stay in walk order.  Two kinds of
        file are indexed alone, in their walk position, once every batch
        before them has been stored (rows in walk order, so get_block's first
        row for a digest is the reference's, src/index.rs:80-90): a FIFO
        (streamed, as index_file streams it) and, with a NativeChunker, a
        regular file of at least `large_file_bytes` (cut on the chunker's
        threads and hashed from one read, sf_index_fd_cut, with the stamp
        taken at its open)."""
        import resource
        from concurrent.futures import ThreadPoolExecutor

        ch = self.chunker
        threads = chunk_threads if chunk_threads > 0 else min(16, os.cpu_count() or 1)
        soft = resource.getrlimit(resource.RLIMIT_NOFILE)[0]
        max_files = max(16, min(4096, (soft if soft > 0 else 1024) // 4))

        def cut(f, stamp):
            sizes = [int(x) for x in ch.fn(f)]
            if sum(sizes) != stamp.size and _stamp_moved(f.fileno(), stamp):
                return None  # written while it was cut
            return _sizes_ok(sizes, stamp.size)

        def finish(batch, futs):
            try:
                cuts = [fu.result() for fu in futs]
                keep = [k for k, c in enumerate(cuts) if c is not None]
                lists = [(_offsets(cuts[k]), np.asarray(cuts[k], np.uint32)) for k in keep]
                res = host.index_fds_blocks([batch[k][3].fileno() for k in keep], lists,
                                            [batch[k][4] for k in keep], stage_bytes=batch_bytes) if keep else None
            finally:
                for _fid, _p, _rel, f, _st in batch:
                    f.close()
            pos = {k: j for j, k in enumerate(keep)}
            for k, (fid, p, rel, _f, _st) in enumerate(batch):
                j = pos.get(k)
                if j is not None and res[3][j] == 0:
                    rows, first, hashes, _status = res
                    self._insert_rows(fid, rows, int(first[j]), int(first[j + 1]))
                    self.db.execute("UPDATE files SET blocks_hash = ? WHERE file_id = ?;",
                                    (bytes(hashes[j]).hex(), fid))
                    continue
                code = SF_EAGAIN if j is None else int(res[3][j])
                if code != SF_EAGAIN:
                    raise SfError(code, f"index_file({os.fsdecode(p)})")
                log.info("File %s changed while it was indexed, indexing it again", p)
                self.db.execute("DELETE FROM blocks WHERE file_id = ?;", (fid,))
                self._index_file_changed(p, rel)

        prev = None
        batch, futs, nbytes = [], [], 0
        native = isinstance(ch, NativeChunker)

        def drain():
            """Store every batch before the file about to be indexed alone."""
            nonlocal prev, batch, futs, nbytes
            if prev is not None:
                p_, prev = prev, None
                finish(*p_)
            if batch:
                b_, f_ = batch, futs
                batch, futs, nbytes = [], [], 0
                finish(b_, f_)

        pool = ThreadPoolExecutor(max_workers=threads)
        try:
            for p, rel in todo:
                f = open(p, "rb")  # File::open first: same error on a missing file
                try:
                    if not _seekable(f):  # a FIFO: read from this open, sequentially, in its place
                        drain()
                        self._index_file_once(p, rel, force=False, opened=f)  # closes f
                        continue
                    stamp = host.file_stamp(f.fileno())
                    file_id, up_to_date = self.add_file(
                        rel, DateTimeUtc.from_ns(stamp.mtime_sec * 10**9 + stamp.mtime_nsec))
                    if not up_to_date and native and stamp.size >= large_file_bytes > 0:
                        drain()
                        try:  # cut on the chunker's threads + hashed, one read of this open
                            rows_np, bh = host.index_fd_cut(f.fileno(), ch.ops, ch.threads or threads, stamp)
                        except SfError as e:
                            if e.code != SF_EAGAIN:
                                raise
                            log.info("File %s changed while it was indexed, indexing it again", p)
                            f.close()
                            self._index_file_changed(p, rel)
                            continue
                        self._insert_rows(file_id, rows_np)
                        self.db.execute("UPDATE files SET blocks_hash = ? WHERE file_id = ?;", (bh.hex(), file_id))
                        f.close()
                        continue
                except BaseException:
                    f.close()
                    raise
                if up_to_date:
                    f.close()
                    continue
                batch.append((file_id, p, rel, f, stamp))
                futs.append(pool.submit(cut, f, stamp))
                nbytes += stamp.size
                if nbytes >= batch_bytes or len(batch) >= max_files:
                    if prev is not None:
                        finish(*prev)  # hashed while the pool cuts this batch
                    prev, batch, futs, nbytes = (batch, futs), [], [], 0
            if prev is not None:
                finish(*prev)
            if batch:
                finish(batch, futs)
        finally:
            pool.shutdown(wait=True)  # no chunker still reading a descriptor closed below
            for b in ([prev[0]] if prev is not None else []) + [batch]:
                for _fid, _p, _rel, f, _st in b:
                    f.close()  # idempotent: the finished batches' are closed already

    def _index_file_changed(self, path, name) -> None:
        """index_file of a file whose first pass saw it change: its row was
        added in walk order already, so only its blocks are indexed again."""
        for attempt in range(CHANGED_RETRIES):
            try:
                self._index_file_once(path, name, force=True)
                return
            except SfError as e:
                if e.code != SF_EAGAIN:
                    raise
        self._index_file_once(path, name, force=True, one_pass=True)

    def _index_batched_boundaries(self, todo, batch_bytes: int) -> None:
        """The default (content-defined) mode over many files: each file is
        read and cut by the host chunker, and the blocks of up to
        `batch_bytes` of files go to the device in ONE sf_index_buffer_blocks
        call (their bytes back to back, one offset-ordered list), so the
        per-call latency of a long block's chain is paid
        per batch, not per file.  Rows get file offsets back; each file's
        blocks_hash is the SHA-1 over its digests in offset order, the value
        compute_blocks_hash reads back (src/index.rs:661-682)."""
        batch = []  # (file_id, base, n_bytes, sizes)
        parts: List[bytes] = []
        nbytes = 0

        def flush():
            nonlocal batch, parts, nbytes
            if not batch:
                return
            offs = np.zeros(sum(len(sz) for _f, _b, _n, sz in batch), np.uint64)
            sizes = np.zeros(offs.size, np.uint32)
            k = 0
            for _fid, base, _n, sz in batch:
                if sz:
                    a = np.asarray(sz, np.uint64)
                    offs[k:k + a.size] = base + np.concatenate([[0], np.cumsum(a)[:-1]]).astype(np.uint64)
                    sizes[k:k + a.size] = a
                    k += a.size
            rows, _ = host.index_buffer_blocks(b"".join(parts), offs, sizes)
            k = 0
            for fid, base, _n, sz in batch:
                mine = rows[k:k + len(sz)].copy()
                k += len(sz)
                mine["offset"] -= np.uint64(base)
                self._insert_rows(fid, mine)
                bh = host.blocks_hash(np.ascontiguousarray(mine["sha1"]))
                self.db.execute("UPDATE files SET blocks_hash = ? WHERE file_id = ?;", (bh.hex(), fid))
            batch, parts, nbytes = [], [], 0

        for p, rel in todo:
            with open(p, "rb") as f:  # File::open first: same error on a missing file
                file_id, up_to_date = self.add_file(rel, _mtime(f))
                if up_to_date:
                    continue
                raw = f.read()  # a FIFO in the tree is read from this open, to EOF
            sizes = _sizes_ok(self.chunker.fn(raw), len(raw))
            batch.append((file_id, nbytes, len(raw), sizes))
            parts.append(raw)
            nbytes += len(raw)
            if nbytes >= batch_bytes:
                flush()
        flush()

    def remove_missing_files(self, path) -> None:
        """src/index.rs:718-726."""
        for file_id, file_path, _m, _s, _bh in self.list_files():
            if not (Path(path) / file_path).is_file():
                log.info("Removing missing file %s", file_path)
                self.remove_file(file_id)
