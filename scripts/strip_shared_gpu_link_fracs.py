#!/usr/bin/env python3
"""Round 5: remove the xGMI fractions from committed collective profiles.

Every collective profile of rounds 1-4 was measured with all ranks on the one
GPU of a gpurun box, so no byte crossed xGMI and a "fraction of xGMI" (up to
1.17 in profiles/r04/bench_n2_shared_gpu_final.json) meant nothing.
bench_collectives.py no longer emits those fields for shared-GPU runs
(msx_engine_gpu_shared); this rewrites the old files the same way: the keys
busbw_frac_xgmi, busbw_frac_measured_links and
xgmi_aggregate_GB_s_per_direction are dropped and the object that held them
is labelled with its plane.  Every other field and value is kept as measured.

usage: scripts/strip_shared_gpu_link_fracs.py profiles/
"""
import json
import os
import sys

DROP = ("busbw_frac_xgmi", "busbw_frac_measured_links", "xgmi_aggregate_GB_s_per_direction")
LABEL = "hbm (ranks shared one GPU; xGMI fractions removed in round 5)"


def strip(o):
    n = 0
    if isinstance(o, dict):
        hit = [k for k in DROP if k in o]
        for k in hit:
            del o[k]
        if hit:
            o.setdefault("plane", LABEL)
            n += len(hit)
        for v in o.values():
            n += strip(v)
    elif isinstance(o, list):
        for v in o:
            n += strip(v)
    return n


def main(root):
    for d, _, files in os.walk(root):
        for f in sorted(files):
            if not f.endswith(".json"):
                continue
            path = os.path.join(d, f)
            text = open(path).read()
            try:
                docs, lines = [json.loads(text)], False
            except json.JSONDecodeError:
                docs = [json.loads(l) if l.strip().startswith("{") else l for l in text.splitlines()]
                lines = True
            n = sum(strip(x) for x in docs if not isinstance(x, str))
            if not n:
                continue
            with open(path, "w") as out:
                if lines:
                    out.write("\n".join(x if isinstance(x, str) else json.dumps(x) for x in docs) + "\n")
                else:
                    json.dump(docs[0], out, indent=1 if "\n" in text.strip() else None)
                    out.write("\n")
            print(f"{path}: {n} fields removed")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "profiles")
