"""Interleaved A/B of kernel variants in ONE process (cdna guide rule 24).

Needs a tuning build of the library (the variants are compiled only with
-DSF_TUNING):  make -C syncfast_amd/csrc variant NAME=tuning EXTRA=-DSF_TUNING
and SF_LIB=syncfast_amd/csrc/build/variants/libsf_tuning.so.

Variants are selected per call through env knobs read by the C-ABI
(SF_VARIANT: 0 shipped = <128,1>, 1 = <128,5>, 2 = <64,6>, 3 = <64,8>, 4 = <64,1>).  Reports median / min ms per launch over rounds and checks that
every variant produces identical digests."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from syncfast_amd import device  # noqa: E402

GiB = 1 << 30


def main():
    size = int(float(os.environ.get("TUNE_GIB", "8")) * GiB)
    bs = int(os.environ.get("TUNE_BS", "4096"))
    variants = [dict(SF_VARIANT=t) for t in os.environ.get("TUNE_VARIANTS", "0,1,2,3,4").split(",")]
    rounds, reps = 5, 5
    data = device.splitmix_tensor(size, 0x5EED0000)
    outs = {}
    times = {str(v): [] for v in variants}
    s = torch.cuda.current_stream()
    for r in range(rounds):
        for v in variants:
            for k, val in v.items():
                os.environ[k] = str(val)
            out = device.index_device(data, bs)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(reps):
                device.index_device(data, bs, out=out)
            e1.record(s)
            torch.cuda.synchronize()
            times[str(v)].append(e0.elapsed_time(e1) / reps)
            if r == 0:
                outs[str(v)] = out.clone()
    ref = next(iter(outs.values()))
    for k, o in outs.items():
        assert torch.equal(o, ref), f"variant {k} digests differ"
    for k, ts in times.items():
        med = statistics.median(ts)
        print(f"{k}: median {med:.4f} ms  min {min(ts):.4f} ms  -> {size / GiB / (med * 1e-3):.1f} GiB/s "
              f"({size * (1 + 20 / bs) / (med * 1e-3) / 1e9:.1f} GB/s alg)", flush=True)


if __name__ == "__main__":
    main()
