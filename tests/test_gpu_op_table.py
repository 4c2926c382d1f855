"""GPU: the builtin op table (MPIR_Op_table, mpid/op.cpp:618-622, entries
MPIR_Op_<op> :703-1923) driven from plain C the way the reference's internal
callers use it: tests/c/op_table_test.c fetches each op's MPI_User_function
with msx_op_table(), calls it on device buffers for every predefined datatype
and compares with the oracle byte for byte; illegal pairs must set op_errno
to MPI_ERR_OP and leave inout untouched (built by __graft_entry__.build())."""
import os
import subprocess

import pytest

import msx

pytestmark = pytest.mark.gpu
REPO = msx.REPO_ROOT
EXE = os.path.join(REPO, "tests", "c", "build", "op_table_test")


def test_op_table_from_c_on_device_buffers():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert os.path.exists(EXE), "build() compiles tests/c first"
    env = dict(os.environ)
    env.pop("MSX_SIZE", None)
    pr = subprocess.run([EXE], capture_output=True, text=True, timeout=240, env=env)
    assert pr.returncode == 0, (pr.stdout + pr.stderr)[-3000:]
    assert pr.stdout.startswith("OK"), pr.stdout
    import oracle
    from _cases import legal_pairs
    legal = int(pr.stdout.split()[1])
    assert legal == len(legal_pairs(oracle)), pr.stdout     # every legal (op, predefined type) pair
