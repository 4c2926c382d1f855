"""GPU: examples/collectives_demo.c, an ordinary MPI program in plain C (gcc,
include/mpi.h, host buffers), run as 1-3 MPI processes on one GPU: reduction
collectives, a user op, a non-blocking allreduce, MPI_Pack of a derived type,
and fence / passive-target one-sided accumulate, each checked exactly inside
the program (exit status 0 on success)."""
import os
import socket
import subprocess

import pytest

import msx

pytestmark = pytest.mark.gpu
REPO = msx.REPO_ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("p", [1, 2, 3])
def test_c_program_collectives(p, tmp_path):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    exe = str(tmp_path / "collectives_demo")
    libdir = os.path.join(REPO, "microsoft-mpi_amd", "lib")
    subprocess.run(["gcc", "-O2", "-Wall", "-Werror", "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "examples", "collectives_demo.c"), "-L", libdir, "-lmsmpi_mi355x",
                    f"-Wl,-rpath,{libdir}", "-o", exe], check=True)
    port = _free_port()
    procs = []
    for r in range(p):
        env = dict(os.environ)
        env.update({"MSX_SIZE": str(p), "MSX_RANK": str(r), "MSX_DEVICE": "0",
                    "MSX_BOOTSTRAP_PORT": str(port), "MSX_BOOTSTRAP_ADDR": "127.0.0.1",
                    "MSX_BOOTSTRAP_TIMEOUT": "120"})
        procs.append(subprocess.Popen([exe], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env))
    for pr in procs:
        try:
            o, e = pr.communicate(timeout=180)
        except subprocess.TimeoutExpired:
            pr.kill()
            o, e = pr.communicate()
        assert pr.returncode == 0, (o + e)[-3000:]
        assert ": OK" in o, o
