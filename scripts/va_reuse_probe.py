"""Coherence after device allocations of another cache type come and go.

One trial: (u) an uncached buffer (hipDeviceMallocUncached, as the engine
windows) written and read by kernels, freed; (nb) a plain buffer written by a
kernel, copied by a kernel into a long-lived buffer V that is checked, freed;
(u2) another uncached buffer, used and freed; the caching allocator emptied;
then torch on a side stream: a = rand(n), b = a.clone(), torch.equal(a, b).
Variants drop or change one step at a time, so the step that matters shows;
the "kept" ones never free the uncached buffers (the library's window pool);
the "host" ones churn page-locked host memory instead (registered in place,
as the library pins a host operand for one call, or hipHostMalloc'd).
A final part checks the engine's own case: pages of a plain buffer reused as an
uncached window written by a kernel and read with plain and non-temporal loads.
Prints one JSON line: per variant, trials, kernel-check failures, torch cases
and torch.equal failures (with details of the first ones).
usage: python scripts/va_reuse_probe.py [trials] [plain]    (GPU only; "plain": the control variant only)"""
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "microsoft-mpi_amd"))
from msx import probe  # noqa: E402

P = probe.lib()
trials = int(sys.argv[1]) if len(sys.argv) > 1 else 32
ONLY_PLAIN = len(sys.argv) > 2 and sys.argv[2] == "plain"   # scripts/va_reuse_xproc.sh
dev = torch.device("cuda:0")
dflt = torch.cuda.default_stream(dev)
sp_d = ctypes.c_void_p(dflt.cuda_stream)
SIZES_MIB = [1, 2, 4, 8]
expect = {}
for mib in SIZES_MIB:
    e = torch.empty(mib << 18, dtype=torch.int32, device=dev)
    assert P.msxp_hbm(probe.WRITE1, None, e.data_ptr(), mib << 20, sp_d) == 0
    expect[mib] = e
V = torch.empty(max(SIZES_MIB) << 18, dtype=torch.int32, device=dev)
scratch = torch.empty(max(SIZES_MIB) << 18, dtype=torch.int32, device=dev)
torch.cuda.synchronize()


KEPT = []
hip = ctypes.CDLL("libamdhip64.so")


def host_churn(nbytes, how):
    """Page-locked host memory read by a kernel, then released: registered in
    place (what the library's pin-for-the-call does with a host operand of
    1 MiB or more) or hipHostMalloc'd."""
    import numpy as np
    if how == "register":
        buf = np.ones(nbytes // 4, dtype=np.int32)
        hp = ctypes.c_void_p(buf.ctypes.data)
        assert hip.hipHostRegister(hp, ctypes.c_size_t(nbytes), 0) == 0
    else:
        hp = ctypes.c_void_p()
        assert hip.hipHostMalloc(ctypes.byref(hp), ctypes.c_size_t(nbytes), 0) == 0
    dp = ctypes.c_void_p()
    assert hip.hipHostGetDevicePointer(ctypes.byref(dp), hp, 0) == 0
    assert P.msxp_hbm(probe.COPY, dp, scratch.data_ptr(), nbytes, sp_d) == 0
    torch.cuda.synchronize()
    if how == "register":
        assert hip.hipHostUnregister(hp) == 0
    else:
        assert hip.hipHostFree(hp) == 0


def churn(nbytes, uncached, read1=True, keep=False):
    u = ctypes.c_void_p()
    assert P.msxp_alloc(nbytes, uncached, ctypes.byref(u)) == 0
    assert P.msxp_hbm(probe.WRITE1, None, u, nbytes, sp_d) == 0
    assert P.msxp_hbm(probe.COPY, u, scratch.data_ptr(), nbytes, sp_d) == 0
    if read1:
        assert P.msxp_hbm(probe.READ1, u, scratch.data_ptr(), nbytes, sp_d) == 0
    torch.cuda.synchronize()
    if keep:
        KEPT.append(u)              # never freed while the process runs (the library's window pool)
    else:
        assert P.msxp_free(u) == 0


def variant(uncached=1, with_u=True, with_nb=True, fresh_side=False, torch_stream="side", keep=False, u_read1=True,
            host=None):
    side = torch.cuda.Stream(dev)
    kfail = tfail = tcases = 0
    details = []
    for t in range(trials):
        mib = SIZES_MIB[t % len(SIZES_MIB)]
        nbytes = mib << 20
        if host:
            host_churn(nbytes, host)
        elif with_u:
            churn(nbytes, uncached, read1=u_read1, keep=keep)
        if with_nb:
            nb = ctypes.c_void_p()
            assert P.msxp_alloc(nbytes, 0, ctypes.byref(nb)) == 0
            V.zero_()
            torch.cuda.synchronize()
            assert P.msxp_hbm(probe.WRITE1, None, nb, nbytes, sp_d) == 0
            assert P.msxp_hbm(probe.COPY, nb, V.data_ptr(), nbytes, sp_d) == 0
            torch.cuda.synchronize()
            kfail += int(int((V[: mib << 18] != expect[mib]).sum()) != 0)
            assert P.msxp_free(nb) == 0
        if host:
            host_churn(nbytes, host)
        else:
            churn(nbytes, uncached, read1=False, keep=keep)
        torch.cuda.empty_cache()
        if fresh_side:
            side = torch.cuda.Stream(dev)
        st = side if torch_stream == "side" else dflt
        with torch.cuda.stream(st):
            for n in (mib << 17, mib << 18, mib << 19):
                a = torch.rand(n, device=dev)
                b = a.clone()
                st.synchronize()
                tcases += 1
                if not torch.equal(a, b):
                    tfail += 1
                    ne1 = int((a != b).sum())
                    torch.cuda.synchronize()
                    ne2 = int((a != b).sum())
                    if len(details) < 6:
                        details.append({"trial": t, "MiB": mib, "n": n, "ne_first": ne1, "ne_after_sync": ne2})
                del a, b
        torch.cuda.synchronize()
    return {"trials": trials, "kernel_check_failures": kfail, "torch_cases": tcases, "torch_equal_failures": tfail,
            "details": details}


summary = {}
for name, kw in (("uncached_full", {}),
                 ("plain_full (control)", {"uncached": 0}),
                 ("uncached_no_u", {"with_u": False}),
                 ("uncached_no_nb", {"with_nb": False}),
                 ("uncached_fresh_side_stream", {"fresh_side": True}),
                 ("uncached_default_stream", {"torch_stream": "default"}),
                 ("uncached_u_without_read1", {"u_read1": False}),
                 ("uncached_full_kept (pool)", {"keep": True}),
                 ("uncached_default_stream_kept (pool)", {"torch_stream": "default", "keep": True}),
                 ("host_register_unregister", {"host": "register"}),
                 ("host_malloc_free", {"host": "malloc"})):
    if ONLY_PLAIN and kw != {"uncached": 0}:
        continue
    summary[name] = variant(**kw)
    print(name, {k: v for k, v in summary[name].items() if k != "details"}, file=sys.stderr, flush=True)

# the engine's own case: pages a plain buffer used (its lines in the L2s) become
# an uncached window; a kernel writes the window (uncached stores, past this
# GPU's L2, like a peer's xGMI writes) and the tree reads it with plain (MTYPE
# UC) and non-temporal loads: a stale L2 line would return the plain data
if ONLY_PLAIN:
    print(json.dumps(summary))
    sys.exit(0)
pv = probe.variants()
PLAIN_LD, NT_LD = pv["u1_b64_plain_rr"], pv["u1_b64_ntld_rr"]
k_fail = k_reuse = 0
for t in range(trials):
    mib = SIZES_MIB[t % len(SIZES_MIB)]
    nbytes = mib << 20
    pb = ctypes.c_void_p()
    assert P.msxp_alloc(nbytes, 0, ctypes.byref(pb)) == 0
    assert P.msxp_hbm(probe.WRITE1, None, pb, nbytes, sp_d) == 0
    for _ in range(2):
        assert P.msxp_hbm(probe.COPY, pb, scratch.data_ptr(), nbytes, sp_d) == 0
        assert P.msxp_variant_run(PLAIN_LD, pb, scratch.data_ptr(), nbytes // 4, sp_d) == 0
    torch.cuda.synchronize()
    pva = pb.value
    assert P.msxp_free(pb) == 0
    ub = ctypes.c_void_p()
    assert P.msxp_alloc(nbytes, 1, ctypes.byref(ub)) == 0
    k_reuse += int(ub.value == pva)
    src = torch.rand(mib << 18, device=dev)
    torch.cuda.synchronize()
    assert P.msxp_hbm(probe.COPY, src.data_ptr(), ub, nbytes, sp_d) == 0
    torch.cuda.synchronize()
    for v in (PLAIN_LD, NT_LD):
        out = torch.zeros(mib << 18, device=dev)
        torch.cuda.synchronize()
        assert P.msxp_variant_run(v, ub, out.data_ptr(), mib << 18, sp_d) == 0     # out = 0 + window
        torch.cuda.synchronize()
        k_fail += int(int((out.view(torch.int32) != src.view(torch.int32)).sum()) != 0)
    assert P.msxp_free(ub) == 0
summary["window_on_reused_plain_pages"] = {"trials": trials, "same_va": k_reuse, "reads": 2 * trials,
                                           "failures": k_fail}
print("window_on_reused_plain_pages", summary["window_on_reused_plain_pages"], file=sys.stderr, flush=True)
for u in KEPT:
    P.msxp_free(u)
print(json.dumps(summary))
