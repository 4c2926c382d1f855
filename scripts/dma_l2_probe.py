"""Does a host-to-device copy (torch .copy_ from a CPU tensor: DMA) leave
stale L2 lines that a kernel on ANOTHER stream reads after a full device
synchronize?  (Round-4 hypothesis for the multirank stress failure, DESIGN.md
§2: a rank's send buffer, reused torch memory, read as its previous zeros by
the library's push kernel.)  Per trial: a buffer is zero-filled and then read
by kernels on torch's stream (so every XCD's L2 may hold its lines), new data
arrives by DMA, torch.cuda.synchronize(), then the library copies the buffer
on its own stream (msx_probe_hbm mode 4, the engine copy kernel) and the copy
is compared with the DMA'd data.  Prints one JSON line with the number of
trials whose copy differed and the first few bad ranges."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "microsoft-mpi_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import msx  # noqa: E402

L = msx.init(errors_return=True)
stream = torch.cuda.Stream()
sp = ctypes.c_void_p(stream.cuda_stream)
trials = int(os.environ.get("TRIALS", "200"))
res = {"trials": 0, "bad_trials": 0, "examples": []}
for nbytes in [int(x) for x in os.environ.get("SIZES", "262144,1200128,4194304").split(",")]:
    x = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    y = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    for t in range(trials):
        x.zero_()                                   # kernel writes: lines in some L2s
        for _ in range(4):
            _ = x.view(torch.int32).sum()           # kernel reads on many CUs / XCDs
        torch.cuda.synchronize()
        host = torch.from_numpy(np.random.default_rng(t).integers(1, 255, nbytes, dtype=np.uint8))
        x.copy_(host)                               # DMA from pageable host memory
        torch.cuda.synchronize()
        y.zero_()
        torch.cuda.synchronize()
        assert L.msx_probe_hbm(4, x.data_ptr(), y.data_ptr(), nbytes, sp) == 0
        torch.cuda.synchronize()
        res["trials"] += 1
        if not torch.equal(y.cpu(), host):
            res["bad_trials"] += 1
            bad = (y.cpu() != host).nonzero().flatten()
            if len(res["examples"]) < 6:
                res["examples"].append({"bytes": nbytes, "trial": t, "n_bad": int(bad.numel()),
                                        "first": int(bad[0]), "last": int(bad[-1]),
                                        "bad_are_zero": bool((y.cpu()[bad] == 0).all())})
    print(json.dumps({nbytes: res}), file=sys.stderr, flush=True)
print(json.dumps(res), flush=True)
