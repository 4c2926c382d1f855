"""GPU: a Fortran program (tests/fortran/f_gpu.f90, built with flang against
include/mpif.h) drives the reduction path through the Fortran bindings
(fortran/mpif.cpp): MPI_REDUCE_LOCAL on host arrays (HIP combine kernels),
MPI_PACK/UNPACK, the blocking and non-blocking reductions with the Fortran
MPI_IN_PLACE / MPI_STATUS_IGNORE / MPI_STATUSES_IGNORE sentinels, a Fortran
user op, and fence-epoch MPI_ACCUMULATE / MPI_FETCH_AND_OP, with 1-3 ranks
sharing one GPU.  Expected values are computed inside the program exactly
(integer data; one IEEE operation per element for the float checks).
"""
import os
import socket
import subprocess

import pytest

import msx

pytestmark = pytest.mark.gpu
REPO = msx.REPO_ROOT
FDIR = os.path.join(REPO, "tests", "fortran")
EXE = os.path.join(FDIR, "build", "f_gpu")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("p", [1, 2, 3])
def test_fortran_program_on_gpu(p):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if not os.path.exists(EXE):
        # normally built by __graft_entry__.build(); flang ships with ROCm
        r = subprocess.run(["make", "-C", FDIR, "build/f_gpu"], capture_output=True, text=True)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    port = _free_port()
    procs = []
    for r in range(p):
        env = dict(os.environ)
        env.update({"MSX_SIZE": str(p), "MSX_RANK": str(r), "MSX_DEVICE": "0",
                    "MSX_BOOTSTRAP_PORT": str(port), "MSX_BOOTSTRAP_ADDR": "127.0.0.1",
                    "MSX_BOOTSTRAP_TIMEOUT": "120"})
        procs.append(subprocess.Popen([EXE], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env))
    results = []
    for pr in procs:
        try:
            o, e = pr.communicate(timeout=180)
        except subprocess.TimeoutExpired:
            pr.kill()
            o, e = pr.communicate()
        results.append((pr.returncode, o, e))
    for rc, o, e in results:
        assert rc == 0, (o + e)[-3000:]
        line = [l for l in o.splitlines() if l.startswith("FRESULT")]
        assert line, (o + e)[-3000:]
        assert line[0].split()[3] == "0", o[-3000:]
