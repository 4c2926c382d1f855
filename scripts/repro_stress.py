"""Replay the multi-rank stress loop of tests/test_gpu_multirank.py with p ranks
sharing ONE GPU, several passes of its 240 calls per process, and report every
rank's RESULT line with the wrong-value diagnosis (stress_diag: zeros, a missing
contribution, a stale contribution from an earlier call, or an earlier result).

Usage: python scripts/repro_stress.py P PASSES [ENV=VALUE ...]
Each rank's output goes to gpurun_out/repro/<tag>/rank<r>.log (progress shows
there and on stdout every 20 s, so a long replay never looks hung).
"""
import os
import socket
import subprocess
import sys
import textwrap
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "microsoft-mpi_amd"))
import test_gpu_multirank as T  # noqa: E402  (the WORKER text, not the tests)


def main():
    p, passes = int(sys.argv[1]), int(sys.argv[2])
    extra = dict(kv.split("=", 1) for kv in sys.argv[3:])
    tag = f"p{p}_x{passes}" + "".join(f"_{k}-{v}" for k, v in extra.items())
    out = os.path.join(REPO, "gpurun_out", "repro", tag)
    os.makedirs(out, exist_ok=True)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs, files = [], []
    for r in range(p):
        env = dict(os.environ)
        env.update({"MSX_SIZE": str(p), "MSX_RANK": str(r), "MSX_DEVICE": "0",
                    "MSX_BOOTSTRAP_PORT": str(port), "MSX_BOOTSTRAP_ADDR": "127.0.0.1",
                    "MSX_BOOTSTRAP_TIMEOUT": "180", "MSX_STRESS_PASSES": str(passes)})
        env.update(extra)
        f = open(os.path.join(out, f"rank{r}.log"), "w")
        files.append(f)
        procs.append(subprocess.Popen([sys.executable, "-u", "-c", f"REPO={REPO!r}\n" + textwrap.dedent(T.WORKER)],
                                      stdout=f, stderr=subprocess.STDOUT, env=env))
    t0 = time.time()
    while any(pr.poll() is None for pr in procs):
        time.sleep(20)
        with open(os.path.join(out, "rank0.log")) as f:
            tail = [l for l in f.read().splitlines() if l.startswith("PASS")]
        print(f"[{time.time() - t0:.0f}s] {tail[-1] if tail else 'prefix'}", flush=True)
    bad = 0
    for r, (pr, f) in enumerate(zip(procs, files)):
        f.close()
        with open(os.path.join(out, f"rank{r}.log")) as g:
            txt = g.read()
        res = [l for l in txt.splitlines() if l.startswith("RESULT")]
        print(f"rank {r} rc={pr.returncode}: {res[0] if res else txt[-800:]}", flush=True)
        bad += pr.returncode != 0 or not res or res[0].split()[3] != "0"
    print(f"{tag}: {bad} rank(s) failed in {time.time() - t0:.0f}s", flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
