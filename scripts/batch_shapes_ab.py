#!/usr/bin/env python3
"""sf_index_device_batch on equal-size files already in HBM, every file's
blocks_hash on the device: the two column halves (SF_BATCH_FUSED=1; the
first run of this script measured round 6's first no-wait form, a fused
launch whose chain slices ran on the last-arriving block wave, at S = 32 and
16) against the block kernel followed by the chain kernel
(SF_BATCH_FUSED=0), over several batch shapes of 8 GiB, interleaved in one
process, HIP events around REPS calls.  With SF_AB_OLD=1 and SF_LIB = round
5's library: its waiting fused launch.  The library is called through raw
ctypes (the Python package binds this round's symbols).  One JSON line per
(shape, form).  Round 6: does the no-wait fused launch earn its keep
?"""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHAPES = [(1024, 8), (256, 32), (64, 128), (16, 512), (4096, 2)]  # files, MiB each: 8 GiB
FORMS = [("halves", 1, None), ("unfused", 0, None)]
if os.environ.get("SF_AB_OLD"):
    FORMS = [("r5_fused_wait", None, None)]


class FileDesc(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_uint64), ("len", ctypes.c_uint64)]


def main():
    import torch
    L = ctypes.CDLL(os.environ.get("SF_LIB") or os.path.join(ROOT, "syncfast_amd", "lib", "libsyncfast_amd.so"))
    vp, u64, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32
    L.sf_index_device_batch.argtypes = [vp, u64, vp, u32, u32, vp, u64, vp, vp, vp, vp, vp]
    L.sf_fill_splitmix_device.argtypes = [vp, u64, u64, u64, vp]
    L.sf_test_set_knob.argtypes = [ctypes.c_char_p, ctypes.c_int64, vp]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    reps, rounds = 5, 4
    data = torch.empty(8 << 30, dtype=torch.uint8, device=dev)
    assert L.sf_fill_splitmix_device(data.data_ptr(), data.numel(), 77, 0, None) == 0
    torch.cuda.synchronize()
    for nf, mib in SHAPES:
        flen = mib << 20
        descs = (FileDesc * nf)(*[FileDesc(i * flen, flen) for i in range(nf)])
        nb = nf * flen // 4096
        dig = torch.empty((nb, 20), dtype=torch.uint8, device=dev)
        fh = torch.empty((nf, 20), dtype=torch.uint8, device=dev)
        st = torch.zeros(1, dtype=torch.int32, device=dev)  # round 5's launch reports a give-up here
        nout = ctypes.c_uint64()

        def call():
            rc = L.sf_index_device_batch(data.data_ptr(), data.numel(), descs, nf, 4096, dig.data_ptr(), nb,
                                         fh.data_ptr(), None, ctypes.byref(nout), st.data_ptr(),
                                         torch.cuda.current_stream().cuda_stream)
            assert rc == 0, rc

        times = {name: [] for name, _f, _s in FORMS}
        ref = None
        for r in range(rounds):
            for name, fused, stages in (FORMS if r % 2 == 0 else FORMS[::-1]):
                if fused is not None:
                    assert L.sf_test_set_knob(b"SF_BATCH_FUSED", fused, None) == 0
                call()  # warm
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    call()
                e1.record()
                torch.cuda.synchronize()
                times[name].append(e0.elapsed_time(e1) / reps)
                assert int(st.item()) == 0, (nf, mib, name, int(st.item()))
                h = fh.cpu().numpy().tobytes()
                assert ref is None or h == ref, (nf, mib, name)
                ref = h
        for name, v in times.items():
            print(json.dumps({"files": nf, "file_mib": mib, "form": name, "ms_median": round(statistics.median(v), 4),
                              "ms_all": [round(x, 4) for x in v], "blocks_hash_0": ref[:20].hex()}), flush=True)


if __name__ == "__main__":
    main()
