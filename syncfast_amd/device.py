"""Device-resident entry points over torch tensors (HBM buffers).

PyTorch is only plumbing here: it owns the HBM allocations and the stream.
Every compute call goes to a HIP kernel through the C-ABI
(``include/syncfast_amd.h``); tensors must live on a ROCm device.

Reference mapping (/root/reference):
  index_device          -> the chunk loop of Index::index_file, src/index.rs:621-647
                           (fixed-size blocks)
  index_device_blocks   -> the same loop for an explicit boundary list
                           (the reference's CDC boundaries, src/index.rs:622-625)
  index_device_batch    -> index_path_rec over many files (src/index.rs:689-715)
                           + compute_blocks_hash per file (src/index.rs:661-682)
"""
from __future__ import annotations

import contextlib
import ctypes
from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from ._lib import FileDesc, check, lib, SF_ERANGE, SfError

__all__ = [
    "num_blocks", "index_device", "index_device_blocks", "index_device_batch",
    "index_device_weak", "index_device_blocks_weak", "BatchStream",
    "fill_splitmix", "splitmix_tensor", "BlockSet", "index_device_multi",
]


def _require_device(t: torch.Tensor, name: str, dtype=None, device: Optional[torch.device] = None) -> None:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.device.type != "cuda":
        raise ValueError(f"{name} must be on a ROCm device (got {t.device}); syncfast_amd has no CPU path")
    if device is not None and t.device != device:
        raise ValueError(f"{name} is on {t.device}, the input on {device}")
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype} (got {t.dtype})")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def _stream_ptr(t: torch.Tensor, stream: Optional[torch.cuda.Stream]) -> int:
    s = stream if stream is not None else torch.cuda.current_stream(t.device)
    return s.cuda_stream


@contextlib.contextmanager
def _on(device: torch.device, stream: Optional[torch.cuda.Stream]):
    """`device` current and, if given, `stream` its current stream: outputs
    and status words are then allocated, zeroed and read back on the stream
    the kernel runs on (a status word zeroed or read on another stream races
    with the kernel that writes it)."""
    with torch.cuda.device(device):
        if stream is None:
            yield
        else:
            with torch.cuda.stream(stream):
                yield


def num_blocks(length: int, block_size: int) -> int:
    """ceil(len / B); 0 for an empty input (no empty blocks)."""
    return (length + block_size - 1) // block_size if length else 0


def index_device(data: torch.Tensor, block_size: int, out: Optional[torch.Tensor] = None,
                 stream: Optional[torch.cuda.Stream] = None) -> torch.Tensor:
    """SHA-1 of every fixed-size block of a uint8 HBM buffer -> uint8[n, 20]."""
    _require_device(data, "data", torch.uint8)
    n = num_blocks(data.numel(), block_size)
    with _on(data.device, stream):
        if out is None:
            out = torch.empty((n, 20), dtype=torch.uint8, device=data.device)
        else:
            _require_device(out, "out", torch.uint8, data.device)
            if out.numel() < 20 * n:
                raise ValueError(f"out holds {out.numel() // 20} digests, need {n}")
        nb = ctypes.c_uint64(0)
        check(lib().sf_index_device_fixed(data.data_ptr() if data.numel() else None, data.numel(),
                                          block_size, out.data_ptr() if n else None, out.numel() // 20,
                                          ctypes.byref(nb), _stream_ptr(data, stream)),
              "sf_index_device_fixed")
    return out


def _blocks_args(data, offsets, sizes):
    _require_device(data, "data", torch.uint8)
    _require_device(offsets, "offsets", torch.int64, data.device)
    _require_device(sizes, "sizes", torch.int32, data.device)
    if sizes.numel() != offsets.numel():
        raise ValueError("offsets and sizes differ in length")
    return offsets.numel()


def index_device_blocks(data: torch.Tensor, offsets: torch.Tensor, sizes: torch.Tensor,
                        out: Optional[torch.Tensor] = None, check_range: bool = True,
                        stream: Optional[torch.cuda.Stream] = None) -> torch.Tensor:
    """SHA-1 of explicit blocks data[offsets[i] : offsets[i] + sizes[i]].

    ``offsets`` int64 and ``sizes`` int32 tensors on the same device.  With
    ``check_range`` a block outside the buffer raises SfError(SF_ERANGE)
    (this synchronises the stream)."""
    n = _blocks_args(data, offsets, sizes)
    with _on(data.device, stream):
        if out is None:
            out = torch.empty((n, 20), dtype=torch.uint8, device=data.device)
        else:
            _require_device(out, "out", torch.uint8, data.device)
            if out.numel() < 20 * n:
                raise ValueError("out too small")
        if n == 0:
            return out
        status = torch.zeros(1, dtype=torch.int32, device=data.device) if check_range else None
        check(lib().sf_index_device_blocks(data.data_ptr() if data.numel() else None, data.numel(),
                                           offsets.data_ptr(), sizes.data_ptr(), n, out.data_ptr(),
                                           status.data_ptr() if status is not None else None,
                                           _stream_ptr(data, stream)),
              "sf_index_device_blocks")
        if status is not None and int(status.item()) != 0:
            raise SfError(SF_ERANGE, "sf_index_device_blocks")
    return out


def index_device_weak(data: torch.Tensor, block_size: int, out: Optional[torch.Tensor] = None,
                      weak_out: Optional[torch.Tensor] = None, stream: Optional[torch.cuda.Stream] = None):
    """index_device plus the opt-in weak sum: (digests uint8[n, 20], weak
    int32[n]) where weak[i] is the zlib Adler-32 of block i (bit pattern of
    the uint32), fused into the same kernel pass.  Not in the reference
    (SURVEY.md 8a row a8)."""
    _require_device(data, "data", torch.uint8)
    n = num_blocks(data.numel(), block_size)
    with _on(data.device, stream):
        if out is None:
            out = torch.empty((n, 20), dtype=torch.uint8, device=data.device)
        if weak_out is None:
            weak_out = torch.empty(n, dtype=torch.int32, device=data.device)
        _require_device(out, "out", torch.uint8, data.device)
        _require_device(weak_out, "weak_out", torch.int32, data.device)
        if out.numel() < 20 * n or weak_out.numel() < n:
            raise ValueError(f"outputs too small for {n} blocks")
        nb = ctypes.c_uint64(0)
        check(lib().sf_index_device_fixed_weak(data.data_ptr() if data.numel() else None, data.numel(), block_size,
                                               out.data_ptr() if n else None, weak_out.data_ptr() if n else None,
                                               min(out.numel() // 20, weak_out.numel()), ctypes.byref(nb),
                                               _stream_ptr(data, stream)),
              "sf_index_device_fixed_weak")
    return out, weak_out


def index_device_blocks_weak(data: torch.Tensor, offsets: torch.Tensor, sizes: torch.Tensor,
                             check_range: bool = True, stream: Optional[torch.cuda.Stream] = None):
    """index_device_blocks plus the opt-in Adler-32 per block (0 for a block
    outside the buffer) -> (digests uint8[n, 20], weak int32[n])."""
    n = _blocks_args(data, offsets, sizes)
    with _on(data.device, stream):
        out = torch.empty((n, 20), dtype=torch.uint8, device=data.device)
        weak = torch.empty(n, dtype=torch.int32, device=data.device)
        if n == 0:
            return out, weak
        status = torch.zeros(1, dtype=torch.int32, device=data.device) if check_range else None
        check(lib().sf_index_device_blocks_weak(data.data_ptr() if data.numel() else None, data.numel(),
                                                offsets.data_ptr(), sizes.data_ptr(), n, out.data_ptr(),
                                                weak.data_ptr(), status.data_ptr() if status is not None else None,
                                                _stream_ptr(data, stream)),
              "sf_index_device_blocks_weak")
        if status is not None and int(status.item()) != 0:
            raise SfError(SF_ERANGE, "sf_index_device_blocks_weak")
    return out, weak


def index_device_batch(data: torch.Tensor, files: Sequence[Tuple[int, int]], block_size: int,
                       file_hashes: bool = True, out: Optional[torch.Tensor] = None,
                       hashes_out: Optional[torch.Tensor] = None, stream: Optional[torch.cuda.Stream] = None,
                       status: Optional[torch.Tensor] = None):
    """Many files inside one HBM buffer.

    ``files`` = [(offset, length), ...].  Returns (digests uint8[n,20],
    first_block int64[n_files+1], file_hashes uint8[n_files,20] or None).

    An equal-size batch with file_hashes runs ONE fused launch in which no
    wave waits (the chains' slices run on the waves that complete their
    dependencies), so nothing can time out.  ``status``
    (int32[1] on the device, may be None) is passed through and is never
    written; it stays for callers of the round-5 interface."""
    _require_device(data, "data", torch.uint8)
    nf = len(files)
    descs = (FileDesc * max(nf, 1))()
    total = 0
    for i, (o, ln) in enumerate(files):
        descs[i].offset, descs[i].len = int(o), int(ln)
        total += num_blocks(int(ln), block_size)
    with _on(data.device, stream):
        if out is None:
            out = torch.empty((total, 20), dtype=torch.uint8, device=data.device)
        else:
            _require_device(out, "out", torch.uint8, data.device)
            if out.numel() < 20 * total:
                raise ValueError("out too small")
        dig = out
        fh = None
        if file_hashes and nf:
            if hashes_out is not None:
                _require_device(hashes_out, "hashes_out", torch.uint8, data.device)
            fh = hashes_out if hashes_out is not None else torch.empty((nf, 20), dtype=torch.uint8, device=data.device)
            if fh.numel() < 20 * nf:
                raise ValueError("hashes_out too small")
        first = np.zeros(nf + 1, np.uint64)
        nb = ctypes.c_uint64(0)
        if status is not None:
            _require_device(status, "status", torch.int32, data.device)
        check(lib().sf_index_device_batch(data.data_ptr() if data.numel() else None, data.numel(), descs, nf,
                                          block_size, dig.data_ptr() if total else None, dig.numel() // 20,
                                          fh.data_ptr() if fh is not None else None,
                                          first.ctypes.data, ctypes.byref(nb),
                                          status.data_ptr() if status is not None else None,
                                          _stream_ptr(data, stream)),
              "sf_index_device_batch")
    return dig, first.astype(np.int64), fh


class BatchStream:
    """Equal-size many-file batches streamed through the device
    (sf_index_device_batch_chained).  Every batch is n_files files of
    file_len bytes back to back in one uint8 HBM tensor.

    push(data, digests) hashes the batch's blocks into `digests` and, in the
    SAME launch, runs the per-file blocks_hash chains of earlier batches:
    with split=True (default) the second half of batch i-2's chains and the
    first half of batch i-1's, so a chain needs only half the latency cover.
    push() returns the blocks_hash tensor (uint8[n_files, 20]) of the batch
    whose chains this launch completes (i-2 split, i-1 unsplit), or None;
    finish() returns the remaining ones in batch order.  push_last(data,
    digests) pushes the stream's last batch and finishes: it returns every
    remaining blocks_hash tensor, and with split chains it hashes that batch
    in two column halves, so the first half of its chains runs beside the
    second half's blocks and only the second half of its chains runs alone.
    A batch's digest table must stay alive until its hashes have been
    returned."""

    def __init__(self, n_files: int, file_len: int, block_size: int, stream: Optional[torch.cuda.Stream] = None,
                 split: bool = True):
        if file_len <= 0 or file_len % block_size:
            raise ValueError("file_len must be a positive multiple of block_size")
        self.n_files, self.file_len, self.block_size = n_files, file_len, block_size
        self.nbf = file_len // block_size
        self.split = split and (self.nbf * 20) // 64 >= 2
        self.stream = stream
        self._b = None  # (digests, hashes): batch waiting for its first half / whole chain
        self._a = None  # (digests, hashes, state): batch waiting for its second half
        self._states = None

    def _job(self, part, entry, state=None):
        from ._lib import ChainJob
        d, h = entry[0], entry[1]
        return ChainJob(d.data_ptr(), self.n_files, part, self.nbf, state.data_ptr() if state is not None else None,
                        h.data_ptr() if part != 1 else None)

    def _launch(self, data, digests, jobs, ref, cols=None):
        from ._lib import ChainJob
        arr = (ChainJob * max(len(jobs), 1))(*jobs)
        lo, hi = cols if cols is not None else (0, self.nbf)
        with _on(ref.device, self.stream):
            check(lib().sf_index_device_batch_chained_cols(
                data.data_ptr() if data is not None else None, self.n_files if data is not None else 0,
                self.file_len, self.block_size, lo, hi, digests.data_ptr() if digests is not None else None,
                arr, len(jobs), _stream_ptr(ref, self.stream)),
                "sf_index_device_batch_chained_cols")

    def _step_jobs(self):
        """Chain jobs for the next launch; advances the pipeline state."""
        jobs, done = [], None
        if self.split:
            if self._a is not None:
                jobs.append(self._job(2, self._a, self._a[2]))
                done = self._a[1]
                self._a = None
            if self._b is not None:
                if self._states is None:
                    dev = self._b[0].device
                    self._states = [torch.empty((self.n_files, 20), dtype=torch.uint8, device=dev) for _ in range(2)]
                st = self._states[0]
                self._states.reverse()  # the next first half writes the other state buffer
                jobs.append(self._job(1, self._b, st))
                self._a = (self._b[0], self._b[1], st)
                self._b = None
        elif self._b is not None:
            jobs.append(self._job(0, self._b))
            done = self._b[1]
            self._b = None
        return jobs, done

    def _check_batch(self, data, digests):
        _require_device(data, "data", torch.uint8)
        _require_device(digests, "digests", torch.uint8, data.device)
        if data.numel() != self.n_files * self.file_len or digests.numel() < 20 * self.n_files * self.nbf:
            raise ValueError("batch or digest table has the wrong size")

    def push(self, data: torch.Tensor, digests: torch.Tensor):
        self._check_batch(data, digests)
        # the chain states and this batch's blocks_hash table are allocated on
        # the stream the launches run on, like every other output here
        with _on(data.device, self.stream):
            jobs, done = self._step_jobs()
            self._launch(data, digests, jobs, data)
            self._b = (digests, torch.empty((self.n_files, 20), dtype=torch.uint8, device=data.device))
        return done

    def _half_cols(self):
        """Column split of a last batch: the first half of every chain (part
        1: bytes [0, 64 * half) of the run) reads digests [0, cut) only."""
        if not self.split or self.nbf % 64 or self.nbf < 128:
            return None
        half = (self.nbf * 20 // 64) // 2  # data chunks of part 1 (as the launcher computes them)
        need = (half * 64 + 19) // 20  # digests part 1 reads
        cut = (need + 63) // 64 * 64  # in whole block waves
        return cut if cut < self.nbf else None

    def push_last(self, data: torch.Tensor, digests: torch.Tensor):
        """Push the stream's last batch and finish; returns every remaining
        blocks_hash tensor in batch order."""
        self._check_batch(data, digests)
        cut = self._half_cols()
        if cut is None:
            done = self.push(data, digests)
            return ([done] if done is not None else []) + self.finish()
        out = []
        with _on(data.device, self.stream):
            # columns [0, cut) beside the jobs push() would run ...
            jobs, done = self._step_jobs()
            self._launch(data, digests, jobs, data, (0, cut))
            if done is not None:
                out.append(done)
            # ... then columns [cut, end) beside the next jobs, which include
            # the first half of this batch's chains (its digests [0, cut) exist)
            self._b = (digests, torch.empty((self.n_files, 20), dtype=torch.uint8, device=data.device))
            jobs, done = self._step_jobs()
            self._launch(data, digests, jobs, data, (cut, self.nbf))
            if done is not None:
                out.append(done)
        return out + self.finish()

    def finish(self):
        out = []
        while self._a is not None or self._b is not None:
            ref = (self._a or self._b)[0]
            with _on(ref.device, self.stream):
                jobs, done = self._step_jobs()
                self._launch(None, None, jobs, ref)
            if done is not None:
                out.append(done)
        return out


class BlockSet:
    """The receiving side's block lookup, on the device (sf_block_set_*).

    Built from a destination index's rows -- ``table`` uint8[n, 20] digests
    in rowid order, ``present`` bool/uint8[n] (None = all present) -- as an
    HBM hash table; ``lookup(digests)`` returns int64[m]: for each digest the
    row of the first present row holding it, or -1.  That is Index::get_block
    (src/index.rs:77-103: hash = ? AND present = 1, SQLite's (hash, rowid)
    order) for a whole FILE_BLOCK list at once, the question
    FsDestinationInner::sink asks per message (src/sync/fs.rs:461-476).
    The set reads ``table`` at lookup time: keep it unchanged while in use."""

    def __init__(self, table: torch.Tensor, present: Optional[torch.Tensor] = None,
                 stream: Optional[torch.cuda.Stream] = None):
        _require_device(table, "table", torch.uint8)
        if table.dim() != 2 or table.shape[1] != 20:
            raise ValueError("table must be uint8[n, 20]")
        n = table.shape[0]
        if present is not None:
            if present.dtype == torch.bool:
                present = present.view(torch.uint8)
            _require_device(present, "present", torch.uint8, table.device)
            if present.numel() != n:
                raise ValueError("present must hold one flag per row")
        self.table, self.present, self.stream = table, present, stream
        self._h = ctypes.c_void_p()
        with _on(table.device, stream):
            check(lib().sf_block_set_build(table.data_ptr() if n else None,
                                           present.data_ptr() if present is not None and n else None, n,
                                           ctypes.byref(self._h), _stream_ptr(table, stream)),
                  "sf_block_set_build")

    def lookup(self, digests: torch.Tensor) -> torch.Tensor:
        _require_device(digests, "digests", torch.uint8, self.table.device)
        if digests.dim() != 2 or digests.shape[1] != 20:
            raise ValueError("digests must be uint8[m, 20]")
        if not self._h:
            raise ValueError("BlockSet is closed")
        m = digests.shape[0]
        with _on(self.table.device, self.stream):
            rows = torch.empty(m, dtype=torch.int64, device=self.table.device)
            if m:
                check(lib().sf_block_set_lookup(self._h, digests.data_ptr(), m, rows.data_ptr(),
                                                _stream_ptr(self.table, self.stream)), "sf_block_set_lookup")
        return rows

    def close(self) -> None:
        if self._h:
            with _on(self.table.device, self.stream):
                check(lib().sf_block_set_free(self._h, _stream_ptr(self.table, self.stream)), "sf_block_set_free")
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def index_device_multi(shards: Sequence[torch.Tensor], file_len: int, block_size: int, root: int = 0,
                       table: Optional[torch.Tensor] = None, scratch: Optional[Sequence[torch.Tensor]] = None,
                       streams: Optional[Sequence[torch.cuda.Stream]] = None,
                       gather_streams: Optional[Sequence[torch.cuda.Stream]] = None) -> torch.Tensor:
    """sf_index_device_multi_ex: shards[r] (on cuda:r) holds shard r
    (host.shard_range) of one logical file; every shard is hashed on its own
    device (on streams[r]) and the digest tables meet in `table` on cuda:root,
    gathered over xGMI with RCCL inside the library (on gather_streams[r],
    after device r's hashing; default: the hash streams).  Returns the
    (nblocks, 20) table, complete once gather_streams[root] (or streams[root])
    has run past the call.  ``streams`` None: each device's default stream.
    The scratch tables and a table allocated here are marked as in use by the
    streams the library reads and writes them on, so the caching allocator
    does not hand them out again before the exchange is done."""
    n = len(shards)
    if n < 1:
        raise ValueError("no shards")
    from .host import shard_range
    nb = num_blocks(file_len, block_size)
    for r, t in enumerate(shards):
        _require_device(t, f"shards[{r}]", torch.uint8, torch.device("cuda", r))
        if t.numel() != shard_range(file_len, block_size, n, r)[1]:
            raise ValueError(f"shards[{r}] is not shard {r} of {n}")
    for name, ss in (("streams", streams), ("gather_streams", gather_streams)):
        if ss is not None and (len(ss) != n or any(s.device != torch.device("cuda", r) for r, s in enumerate(ss))):
            raise ValueError(f"{name}[r] must be a stream of cuda:r, one per shard")
    hs = list(streams) if streams is not None else [torch.cuda.default_stream(r) for r in range(n)]
    gs = list(gather_streams) if gather_streams is not None else hs
    dev_root = torch.device("cuda", root)
    own_table = table is None
    if own_table:
        table = torch.empty((max(nb, 1), 20), dtype=torch.uint8, device=dev_root)
    _require_device(table, "table", torch.uint8, dev_root)
    if table.numel() < nb * 20:
        raise ValueError("table too small")
    own_scratch = scratch is None
    if own_scratch:
        scratch = [torch.empty((max(num_blocks(t.numel(), block_size), 1), 20), dtype=torch.uint8, device=t.device)
                   for t in shards]
    ptr = lambda ts: (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts])  # noqa: E731
    sp = (ctypes.c_void_p * n)(*[s.cuda_stream for s in hs])
    gp = (ctypes.c_void_p * n)(*[s.cuda_stream for s in gs])
    check(lib().sf_index_device_multi_ex(n, ptr(shards), file_len, block_size, ptr(scratch), root, table.data_ptr(),
                                         sp, gp), "sf_index_device_multi_ex")
    if own_scratch:  # device r's scratch is written on hs[r] and sent on gs[r]
        for r in range(n):
            for st in {hs[r], gs[r]}:
                scratch[r].record_stream(st)
    if own_table:  # the root's rows are written on hs[root], the others received on gs[root]
        for st in {hs[root], gs[root]}:
            table.record_stream(st)
    return table[:nb]


def fill_splitmix(out: torch.Tensor, seed: int, start: int = 0,
                  stream: Optional[torch.cuda.Stream] = None) -> torch.Tensor:
    """Fill a uint8 HBM buffer with bytes [start, start+len) of the
    splitmix64 stream `seed` (the synthetic input of bench.py / tests)."""
    _require_device(out, "out", torch.uint8)
    with torch.cuda.device(out.device):
        check(lib().sf_fill_splitmix_device(out.data_ptr() if out.numel() else None, out.numel(),
                                            seed & 0xFFFFFFFFFFFFFFFF, start, _stream_ptr(out, stream)),
              "sf_fill_splitmix_device")
    return out


def splitmix_tensor(length: int, seed: int, device="cuda", start: int = 0) -> torch.Tensor:
    t = torch.empty(length, dtype=torch.uint8, device=device)
    return fill_splitmix(t, seed, start)
