"""The list pipeline's stage size for one mid-size file (configs[0]'s 64 MiB,
the default mode's hashing call after sf_cut_fd): sf_index -Z -p 16 -T with
SF_TEST_STREAM_STAGE_MIB = 256 (the default) / 64 / 32 / 16, interleaved,
REPS rounds; the best of the three in-process passes per run."""
import json
import os
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import oracle  # noqa: E402  (input bytes only)

EXE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "examples", "build", "sf_index")


def main():
    reps = int(os.environ.get("REPS", "5"))
    stages = [int(x) for x in os.environ.get("STAGES", "256,64,32,16").split(",")]
    d = tempfile.mkdtemp(prefix="sf_stage_")
    p = os.path.join(d, "f64m")
    oracle.splitmix_bytes(64 << 20, 0x5EED0000).tofile(p)
    try:
        for r in range(reps):
            for sm in stages[r % len(stages):] + stages[:r % len(stages)]:
                env = dict(os.environ, SF_TEST_STREAM_STAGE_MIB=str(sm))
                out = subprocess.run([EXE, "-Z", "-p", "16", "-T", p, p, p], capture_output=True, text=True, env=env,
                                     timeout=120)
                t = [json.loads(ln) for ln in out.stderr.splitlines() if ln.startswith("{")]
                best = min(t[1:], key=lambda x: x["chunk_s"] + x["hash_s"])
                print(json.dumps({"rep": r, "stage_mib": sm, "chunk_ms": round(best["chunk_s"] * 1e3, 3),
                                  "hash_ms": round(best["hash_s"] * 1e3, 3),
                                  "e2e_GB/s": round((64 << 20) / (best["chunk_s"] + best["hash_s"]) / 1e9, 3)}),
                      flush=True)
    finally:
        os.unlink(p)
        os.rmdir(d)


if __name__ == "__main__":
    main()
