"""torch.equal / eq().all() against ne().sum() / ne().any() on equal tensors,
on the default stream and on a side stream set with torch.cuda.set_stream, at
several sizes; no msx code involved.  Prints one line per case whose answers
disagree and a JSON summary.
usage: python scripts/torch_equal_probe.py    (GPU only)"""
import json
import sys

import torch

dev = torch.device("cuda:0")
side = torch.cuda.Stream(dev)
bad = []
cases = 0
for stream_kind in ("default", "side"):
    if stream_kind == "side":
        torch.cuda.set_stream(side)
    for log2n in range(16, 25):
        n = 1 << log2n
        for rep in range(3):
            a = torch.rand(n, device=dev)
            b = a.clone()
            torch.cuda.synchronize()
            r = {"equal": torch.equal(a, b), "equal_i32": torch.equal(a.view(torch.int32), b.view(torch.int32)),
                 "eq_all": bool(torch.eq(a, b).all()), "ne_sum0": int((a != b).sum()) == 0,
                 "ne_any_not": not bool((a != b).any())}
            cases += 1
            if not all(r.values()):
                bad.append({"stream": stream_kind, "n": n, "rep": rep, **r})
                print("DISAGREE", bad[-1], file=sys.stderr, flush=True)
torch.cuda.set_stream(torch.cuda.default_stream(dev))
print(json.dumps({"torch": torch.__version__, "cases": cases, "disagreements": bad}))
