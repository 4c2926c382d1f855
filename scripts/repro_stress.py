"""Replay the multi-rank stress loop of tests/test_gpu_multirank.py with p ranks
sharing ONE GPU, several passes of its 240 calls per process, and report every
rank's RESULT line with the wrong-value diagnosis (stress_diag: zeros, a missing
contribution, a stale contribution from an earlier call, or an earlier result).

Usage: python scripts/repro_stress.py P PASSES [ENV=VALUE ...]
Each rank's output goes to gpurun_out/repro/<tag>/rank<r>.log (progress shows
there and on stdout every 20 s, so a long replay never looks hung).

REPRO_PARENT_QUEUES=k (k > 0): this parent process first opens the GPU and runs
a kernel on k streams, so it holds hardware queues while the ranks run, as the
pytest parent does in a whole-suite run (its own in-process GPU tests ran
before the multirank ones).  REPRO_PARENT_BUSY=1: it also keeps launching small
kernels on those streams until the ranks end, so the queue scheduler has to
time-slice more queues than the GPU maps at once.
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
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    # parent settings, from the command line (not passed on to the ranks)
    pq = int(extra.pop("REPRO_PARENT_QUEUES", os.environ.get("REPRO_PARENT_QUEUES", "0")))
    busy = extra.pop("REPRO_PARENT_BUSY", os.environ.get("REPRO_PARENT_BUSY", "0")) == "1"
    tag = f"p{p}_x{passes}" + "".join(f"_{k}-{v}" for k, v in extra.items())
    out = os.path.join(REPO, "gpurun_out", "repro", tag)
    if pq > 0:
        import torch
        streams = [torch.cuda.Stream() for _ in range(pq)]
        bufs = []
        for st in streams:
            with torch.cuda.stream(st):
                bufs.append(torch.ones(1 << 20, device="cuda"))
                bufs[-1].mul_(1.0001)
        torch.cuda.synchronize()
        tag += f"_parentq{pq}" + ("_busy" if busy else "")
        out = os.path.join(REPO, "gpurun_out", "repro", tag)
    os.makedirs(out, exist_ok=True)
    procs, files = [], []
    for r in range(p):
        env = dict(os.environ)
        env.update({"MSX_SIZE": str(p), "MSX_RANK": str(r), "MSX_DEVICE": "0",
                    "MSX_BOOTSTRAP_PORT": str(port), "MSX_BOOTSTRAP_ADDR": "127.0.0.1",
                    "MSX_BOOTSTRAP_TIMEOUT": "180", "MSX_STRESS_PASSES": str(passes)})
        env.setdefault("MSX_TWO_STEP_MAX", str(1 << 62))   # the GPU-flag schedules the round-3 failure ran
        env.update(extra)
        f = open(os.path.join(out, f"rank{r}.log"), "w")
        files.append(f)
        procs.append(subprocess.Popen([sys.executable, "-u", "-c", f"REPO={REPO!r}\n" + textwrap.dedent(T.WORKER)],
                                      stdout=f, stderr=subprocess.STDOUT, env=env))
    t0 = time.time()
    launches = 0
    while any(pr.poll() is None for pr in procs):
        if pq > 0 and busy:
            t1 = time.time()
            while time.time() - t1 < 20 and any(pr.poll() is None for pr in procs):
                for st, b in zip(streams, bufs):
                    with torch.cuda.stream(st):
                        b.mul_(1.0001)
                launches += len(streams)
                if launches % 256 < len(streams):
                    torch.cuda.synchronize()
            torch.cuda.synchronize()
        else:
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
    print(f"{tag}: {bad} rank(s) failed in {time.time() - t0:.0f}s (parent launches {launches})", flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
