#!/usr/bin/env python3
"""bench.py — headline benchmark of the MI355X MS-MPI reduction path.

Metric (BASELINE.json): GiB/s of a device-resident MPI_SUM local reduce over
MPI_FLOAT, 256 MiB per operand per GPU (config 2), at 1/2/4/8 GPUs, and the
fraction of the HBM roofline.

* A "step" is one MPI_SUM combine `inout[i] += in[i]` over the whole 256 MiB
  buffers (67,108,864 fp32), issued through the C ABI msx_reduce_local_dev
  (the device entry point of MPI_Reduce_local) on one HIP stream, inputs
  already resident in HBM.
* `value` = whole-job HBM traffic rate: ranks x steps x 12 B/element (two 4-B
  reads + one 4-B write) / max-over-ranks wall time, in GiB/s.  The payload
  rate (4 B/element) is reported beside it.
* N > 1: one process per GPU (torchrun), each rank reduces its own shard
  (weak scaling, no data-path collective: the elements are independent).
* roofline: algorithmic bytes per launch / mean kernel duration from HIP
  events on the launch stream, against 8 TB/s (MI355X_MICROARCH.md).
  `traffic` comes from the committed rocprofv3 PMC summary (FETCH_SIZE
  doubled per the gfx950 calibration + WRITE_SIZE) when present.
* cpu_baseline: the oracle (C restatement of op.cpp's Op<float>::Sum) timed
  on this host, one thread = one MS-MPI rank, on a bounded sample.
* N > 1 also runs the collective configs c3-c5 (bench_collectives.py) in
  child processes, headline configs first, every child under a time limit cut
  to what is left of one wall budget (MSX_BENCH_WALL_S, default 420 s from
  process start), so one hung data plane can never cost the JSON line.
* The HBM probes, the combine variants of --sweep and the cold-cache launches
  run the bench-only measurement kernels of libmsx_probe.so (msx.probe); the
  timed steps run the product library's msx_reduce_local_dev.
"""
import argparse
import ctypes
import glob
import json
import os
import sys
import time

T_START = time.time()          # the wall budget of the N > 1 children counts from here
REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "microsoft-mpi_amd"))

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
N_ELEM = 64 << 20              # 256 MiB of fp32 per operand (config 2)
BYTES_PER_ELEM = 12            # 2 x 4 B read + 4 B write
HOST_SIZES = (8, 4 << 10, 64 << 10, 1 << 20, 16 << 20, 256 << 20)   # host-operand crossover table


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--sweep", action="store_true",
                    help="time the probe library's combine variants next to the product kernel (rank 0 stderr)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-host-path", action="store_true")
    ap.add_argument("--elems", type=int, default=N_ELEM)
    ap.add_argument("--no-collectives", action="store_true",
                    help="skip the N>1 collective configs (c3-c5, bench_collectives.py)")
    ap.add_argument("--coll-scale", type=float, default=1.0, help="size factor for c3-c5")
    ap.add_argument("--no-per-op", action="store_true", help="skip the per-(op, type) roofline table")
    ap.add_argument("--no-pack", action="store_true", help="skip the datatype pack/unpack table")
    ap.add_argument("--rccl-native-child", metavar="OUT", help=argparse.SUPPRESS)
    ap.add_argument("--multi-host-child", metavar="OUT", help=argparse.SUPPRESS)
    return ap.parse_args()


# The N > 1 children share one wall budget (from process start, rank 0's
# clock): each runs under min(its own ceiling, what is left minus a reserve
# for the cold-cache launch, the JSON line and teardown), and is skipped when
# less than MIN_CHILD_S would be left.  Worst case with every child hanging:
# the budget itself.  Order: the IPC plane's c3-c5 (the default data plane),
# the RCCL planes' c3-c5, RCCL's own allreduce, the engine variant, then the
# IPC plane's remaining configs and the host-memory multi-GPU split.
WALL_BUDGET_S = float(os.environ.get("MSX_BENCH_WALL_S", "420"))
RESERVE_S = 25.0
MIN_CHILD_S = 20.0
CHILD_CAP_S = {"ipc_core": 150.0, "rccl_core": 120.0, "rccl_native_core": 120.0, "rccl_allreduce": 90.0,
               "variant_pipeline": 120.0, "ipc_extras": 150.0, "multi_host": 60.0}

CHILD_ORDER = ("ipc_core", "rccl_core", "rccl_native_core", "rccl_allreduce", "variant_pipeline", "ipc_extras",
               "multi_host")


def child_timeout(name, elapsed_s):
    """Seconds child `name` may run when `elapsed_s` of the wall budget are
    gone, or None when it is skipped (less than MIN_CHILD_S left)."""
    t = min(CHILD_CAP_S[name], WALL_BUDGET_S - elapsed_s - RESERVE_S)
    return t if t >= MIN_CHILD_S else None


# c3 / c4 under the other schedule at N = 8 (one GPU per rank): the GPU-flag
# pipeline at every size, where the default takes the host-barrier schedule
# above 256 MiB (DESIGN.md §4's decision rule reads the two against each other)
C3_VARIANTS = (("pipeline", {"MSX_TWO_STEP_MAX": str(1 << 62)}),)


def run_collectives_child(world, rank, local, scale, transport="ipc", extra_env=None, tag="", port_off=0,
                          parts="all", timeout=150.0):
    """c3-c5 in a child MPI process per rank (isolated from the headline line).
    transport "ipc": IPC windows + xGMI remote writes; "rccl": RCCL send/recv;
    "rccl_native": RCCL's own collectives where the (op, type) pair maps.
    parts: bench_collectives.py's MSX_COLL_PARTS.  The child is killed after
    `timeout` seconds."""
    import subprocess
    import tempfile
    out = os.path.join(tempfile.gettempdir(),
                       f"msx_coll_{transport}{tag}_{parts}_{os.environ.get('MASTER_PORT', '0')}.json")
    env = dict(os.environ)
    env.update(extra_env or {})
    env["MSX_COLL_PARTS"] = parts
    off = {"ipc": 113, "rccl": 127, "rccl_native": 139}[transport] + port_off   # same on every rank
    env.update({"MSX_SIZE": str(world), "MSX_RANK": str(rank), "MSX_DEVICE": str(local),
                "MSX_TRANSPORT": transport,
                "MSX_BOOTSTRAP_ADDR": os.environ.get("MASTER_ADDR", "127.0.0.1"),
                "MSX_BOOTSTRAP_PORT": str((int(os.environ.get("MASTER_PORT", "29500")) + off) % 65536),
                "MSX_BOOTSTRAP_TIMEOUT": "90", "MSX_STUCK_SYNC_S": "60",
                "MSX_BENCH_LOG": os.environ.get("MSX_BENCH_LOG", os.devnull)})
    mine = f"{out}.rank{rank}"
    for path in (out, mine):
        if os.path.exists(path):
            os.remove(path)

    def child_error(what, stderr):
        """The child's own structured error (bench_collectives.fail), else the
        library's MSX_STUCK reports (rank, phase, peer of a blocked step)."""
        try:
            with open(mine) as f:
                err = json.load(f).get("error")
            if err:
                return err
        except (OSError, ValueError):
            pass
        stuck = []
        for line in (stderr or "").splitlines():
            if line.startswith("MSX_STUCK "):
                try:
                    stuck.append(json.loads(line[len("MSX_STUCK "):]))
                except ValueError:
                    pass
        err = {"rank": rank, "text": f"child {what}: {(stderr or '')[-400:]}"}
        if stuck:
            err.update({"kind": "stuck", "phase": stuck[-1].get("phase"), "peer": stuck[-1].get("peer"),
                        "stuck": stuck[-4:]})
        return err

    try:
        pr = subprocess.run([sys.executable, os.path.join(REPO, "bench_collectives.py"), out, str(scale)],
                            env=env, capture_output=True, text=True, timeout=timeout)
        if pr.returncode != 0:
            return {"error": child_error(f"rc={pr.returncode}", pr.stderr)}
    except subprocess.TimeoutExpired as e:
        se = e.stderr.decode(errors="replace") if isinstance(e.stderr, bytes) else e.stderr
        return {"error": child_error(f"timed out after {timeout:.0f} s", se)}
    if rank == 0:
        try:
            with open(out) as f:
                return json.load(f)
        except OSError as e:
            return {"error": str(e)}
    return {}


class stdout_to_stderr:
    """fd-level redirect: gloo/RCCL print connection chatter on stdout, which
    must carry nothing but rank 0's JSON line."""
    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def rccl_native_child_main(out, scale):
    """Child-process body of rccl_native_allreduce: its own torch.distributed
    job (backend "nccl" = RCCL) on this rank's GPU; rank 0 writes the JSON."""
    import torch
    import torch.distributed as dist
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    local = int(os.environ["LOCAL_RANK"]) % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", init_method="env://", device_id=torch.device("cuda", local))
    n = int((1 << 28) * scale)
    x = torch.ones(n, device="cuda")
    for _ in range(2):
        dist.all_reduce(x)
    torch.cuda.synchronize()
    dist.barrier()
    reps, t0 = 5, time.perf_counter()
    for _ in range(reps):
        dist.all_reduce(x)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    t = torch.tensor([dt], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    ok = bool(torch.all(x == float(world) ** (reps + 2)).item())
    if rank == 0:
        alg = n * 4 / dt / 1e9
        with open(out, "w") as f:
            json.dump({"bytes_per_rank": n * 4, "seconds": round(dt, 5), "algbw_GB_s": round(alg, 2),
                       "busbw_GB_s": round(alg * 2 * (world - 1) / world, 2), "correct": ok}, f)
    dist.destroy_process_group()


def rccl_native_allreduce(world, rank, local, scale, timeout=90.0):
    """xGMI reference point: RCCL's own fp32 SUM allreduce (its ring/tree order,
    NOT the reference's association) on c3's 1 GiB/rank, same GPUs.  Runs in a
    child process per rank with its own rendezvous and a time limit, so an
    RCCL failure or hang is reported in the JSON line and never stalls it."""
    import subprocess
    import tempfile
    out = os.path.join(tempfile.gettempdir(), f"msx_rccl_native_{os.environ.get('MASTER_PORT', '0')}.json")
    env = dict(os.environ)
    env.update({"MASTER_PORT": str((int(os.environ.get("MASTER_PORT", "29500")) + 131) % 65536),
                "RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(local)})
    try:
        pr = subprocess.run([sys.executable, os.path.abspath(__file__), "--rccl-native-child", out,
                             "--coll-scale", str(scale)], env=env, capture_output=True, text=True,
                            timeout=timeout)
        if pr.returncode != 0:
            return {"error": f"rank {rank} child rc={pr.returncode}: {pr.stderr[-600:]}"}
    except subprocess.TimeoutExpired:
        return {"error": f"rank {rank} child timed out after {timeout:.0f} s"}
    if rank == 0:
        try:
            with open(out) as f:
                return json.load(f)
        except (OSError, ValueError) as e:
            return {"error": str(e)}
    return {}


def multi_host_child_main(out, n):
    """Child body of run_multi_host_child: one process, every visible GPU."""
    import numpy as np
    import torch
    import msx
    os.environ["MSX_SIZE"], os.environ["MSX_RANK"] = "1", "0"
    L = msx.init(errors_return=True)
    C = msx.C
    ngpu = torch.cuda.device_count()
    ha = np.random.default_rng(1).uniform(-1, 1, n).astype(np.float32)
    hb = np.random.default_rng(2).uniform(-1, 1, n).astype(np.float32)
    exp = hb + ha
    res = {"bytes_per_operand": n * 4, "gpus_visible": ngpu, "host_memory": "pageable",
           "api": "msx_reduce_local_multi (pinned for the call, each GPU over its own PCIe link)"}
    for g in sorted({1, ngpu}):
        hb2 = hb.copy()
        rc = L.msx_reduce_local_multi(ha.ctypes.data, hb2.ctypes.data, n, C.MPI_FLOAT, C.MPI_SUM, g)
        ok = rc == 0 and hb2.tobytes() == exp.tobytes()
        ts = []
        for _ in range(3):
            t1 = time.perf_counter()
            L.msx_reduce_local_multi(ha.ctypes.data, hb2.ctypes.data, n, C.MPI_FLOAT, C.MPI_SUM, g)
            ts.append(time.perf_counter() - t1)
        t = sorted(ts)[1]
        res[f"{g}_gpu"] = {"ms_per_call": round(t * 1e3, 2), "payload_GiB_s": round(n * 4 / t / 2**30, 2),
                           "correct_first_call": ok}
    with open(out, "w") as f:
        json.dump(res, f)


def run_multi_host_child(n, timeout=60.0):
    import subprocess
    import tempfile
    out = os.path.join(tempfile.gettempdir(), f"msx_multi_host_{os.getpid()}.json")
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MSX_DEVICE"):
        env.pop(k, None)
    try:
        pr = subprocess.run([sys.executable, os.path.abspath(__file__), "--multi-host-child", out,
                             "--elems", str(n)], env=env, capture_output=True, text=True, timeout=timeout)
        if pr.returncode != 0:
            return {"error": f"child rc={pr.returncode}: {pr.stderr[-600:]}"}
        with open(out) as f:
            return json.load(f)
    except subprocess.TimeoutExpired:
        return {"error": f"child timed out after {timeout:.0f} s"}
    except (OSError, ValueError) as e:
        return {"error": str(e)}


class ChildRunners:
    """The N > 1 child processes run_children starts (tests substitute fakes)."""
    collectives = staticmethod(run_collectives_child)
    rccl_allreduce = staticmethod(rccl_native_allreduce)
    multi_host = staticmethod(run_multi_host_child)


def run_children(dist, world, rank, local, scale, n, distinct, no_host_path, runners=ChildRunners):
    """The collective configs and the node-level host split at N > 1, in child
    processes, each under a time limit cut to the remaining wall budget
    (WALL_BUDGET_S, CHILD_ORDER); rank 0's clock decides, so every rank runs
    and skips the same children.  Collective over `dist` (every rank calls
    it); returns rank 0's results (other ranks: their own, unused).
    distinct: one GPU per rank (the RCCL planes need it)."""
    import torch
    coll = coll_rccl = coll_native = rccl_native = c3_variants = coll_extras = multi_host = None
    budget = {"wall_budget_s": WALL_BUDGET_S, "reserve_s": RESERVE_S, "child_cap_s": CHILD_CAP_S, "steps": []}

    def allot(name, collective=True):
        """Seconds child `name` may run (None: skipped), from rank 0's clock."""
        el = [time.time() - T_START]
        if collective:
            dist.broadcast_object_list(el, src=0)
        t = child_timeout(name, el[0])
        step = {"name": name, "start_s": round(el[0], 1), "timeout_s": None if t is None else round(t, 1)}
        if t is None:
            step["skipped"] = "wall budget"
        budget["steps"].append(step)
        return t

    def took(res):
        budget["steps"][-1]["elapsed_s"] = round(time.time() - T_START - budget["steps"][-1]["start_s"], 1)
        if isinstance(res, dict) and "error" in res:
            budget["steps"][-1]["error"] = True
        return res

    def collect(transport, name, parts, extra=None, tag="", port_off=0):
        t = allot(name)
        if t is None:
            return {"skipped": "wall budget"} if rank == 0 else None
        mine = runners.collectives(world, rank, local, scale, transport, extra, tag, port_off,
                                     parts=parts, timeout=t)
        errs = [None] * world
        dist.all_gather_object(errs, mine.get("error"))      # every rank's structured error
        res = mine if rank == 0 else None
        if rank == 0 and any(e is not None for e in errs):
            res["errors"] = [dict(e, rank=r) if isinstance(e, dict) else {"rank": r, "text": e}
                             for r, e in enumerate(errs) if e is not None]
            res.setdefault("error", res["errors"][0])
        return took(res) if rank == 0 else None
    # 1. the default data plane's headline configs (and the all-peer probe)
    coll = collect("ipc", "ipc_core", "core")
    if distinct:
        # 2. the RCCL send/recv plane, then this library's MPI calls on
        # RCCL's own collectives (MSX_TRANSPORT=rccl_native: ncclAllReduce /
        # ncclReduce / ncclReduceScatter where the pair maps, RCCL order;
        # the harness's integer-valued inputs make every order exact, so
        # `correct` still checks in full)
        coll_rccl = collect("rccl", "rccl_core", "core")
        coll_native = collect("rccl_native", "rccl_native_core", "core")
        # 3. RCCL's own fp32 allreduce (torch.distributed), the xGMI reference point
        t = allot("rccl_allreduce")
        if t is not None:
            mine = runners.rccl_allreduce(world, rank, local, scale, timeout=t)
            ok = torch.tensor([0 if "error" in mine else 1], dtype=torch.int32)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            rccl_native = mine if rank == 0 else None
            if rank == 0:
                if not ok.item() and "error" not in rccl_native:
                    rccl_native["error"] = "a non-zero rank's child failed"
                took(rccl_native)
    # 4. the other schedule of c3 / c4 (IPC plane) at N = 8, or at the N
    # that MSX_BENCH_VARIANTS_AT names (a rehearsal on fewer GPUs); skipped
    # when the default IPC run failed (it would only repeat the failure)
    ipc_failed = [rank == 0 and (coll is None or "error" in coll or "skipped" in coll)]
    dist.broadcast_object_list(ipc_failed, src=0)
    if world == int(os.environ.get("MSX_BENCH_VARIANTS_AT", "8")):
        if ipc_failed[0]:
            c3_variants = {"skipped": "the default IPC collectives child failed (see collectives.error)"}
        else:
            c3_variants = {}
            for vi, (name, extra) in enumerate(C3_VARIANTS):
                mine = collect("ipc", "variant_" + name, "c3c4", extra, tag="_" + name, port_off=200 + 11 * vi)
                if rank == 0:
                    ent = {"env": extra}
                    if "skipped" in mine:
                        ent["skipped"] = mine["skipped"]
                    for key, tag in (("c3_allreduce_sum_f32", "c3"), ("c4_reduce_scatter_max_f64", "c4")):
                        v = mine.get(key) or {}
                        ent[tag] = {k: v.get(k) for k in ("seconds", "busbw_GB_s", "correct") if k in v}
                    if mine.get("errors"):
                        ent["errors"] = mine["errors"]
                    c3_variants[name] = ent
    # 5. the IPC plane's remaining configs (curve, host memory, rooted
    # reduce, scan, one-sided accumulate)
    coll_extras = collect("ipc", "ipc_extras", "extras", tag="_extras", port_off=300)
    # 6. SURVEY §8(e) strong-scaled local reduce on the MPI path's host
    # buffers: one 256 MiB fp32 MPI_SUM vector split over every GPU of the
    # node, each GPU over its own PCIe link (msx_reduce_local_multi),
    # against the same call on one GPU -- rank 0 only, while the other
    # ranks wait at the closing barrier
    if rank == 0 and not no_host_path:
        t = allot("multi_host", collective=False)
        multi_host = took(runners.multi_host(n, timeout=t)) if t is not None else {"skipped": "wall budget"}
    return {"coll": coll, "coll_rccl": coll_rccl, "coll_native": coll_native, "rccl_native": rccl_native,
            "c3_variants": c3_variants, "coll_extras": coll_extras, "multi_host": multi_host, "budget": budget,
            "distinct": distinct}


def collectives_report(kids):
    """Rank 0's JSON fields for run_children's results: per data plane, c3-c5
    correct / busBW and the fraction of the links' measured rate (the IPC
    child's all-peer write probe: every GPU writing into all peers' windows at
    once); null fractions when the ranks share a GPU (no byte crosses xGMI)
    or the probe did not run."""
    coll, coll_rccl, coll_native = kids["coll"], kids["coll_rccl"], kids["coll_native"]
    rccl_native, budget = kids["rccl_native"], kids["budget"]
    out = {}
    shared = not kids["distinct"] or bool(coll and coll.get("gpu_shared"))
    links = None if shared else ((coll or {}).get("peer_write_probe") or {}).get("outbound_GB_s_per_gpu")

    def summarize(c):
        if not c:
            return None
        sm = {}
        for key, tag in (("c3_allreduce_sum_f32", "c3"), ("c4_reduce_scatter_max_f64", "c4"),
                         ("c5_iallreduce_band_u64", "c5")):
            v = c.get(key)
            if v:
                sm[tag] = {k: v.get(k) for k in ("correct", "busbw_GB_s", "seconds", "t_comm_s") if k in v}
                bw = v.get("busbw_GB_s")
                sm[tag]["busbw_frac_measured_links"] = round(bw / links, 3) if (bw and links) else None
        for k in ("error", "skipped"):
            if k in c:
                sm[k] = c[k]
        return sm
    if coll is not None or coll_rccl is not None:
        native = None
        if rccl_native is not None:
            bw = rccl_native.get("busbw_GB_s")
            native = {k: rccl_native.get(k) for k in ("correct", "busbw_GB_s", "error", "skipped") if k in rccl_native}
            native["busbw_frac_measured_links"] = round(bw / links, 3) if (bw and links) else None
        out["collectives_summary"] = {"plane": "hbm (ranks share one GPU)" if shared else "xgmi",
                                      "measured_links_GB_s_per_gpu": links,
                                      "ipc": summarize(coll), "rccl": summarize(coll_rccl),
                                      "rccl_native": summarize(coll_native),
                                      "rccl_own_allreduce_f32": native}
    if budget["steps"]:
        budget["wall_s_at_json"] = round(time.time() - T_START, 1)
        out["wall_budget"] = budget
    for key, name in (("coll_extras", "collectives_extras"), ("coll", "collectives"),
                      ("coll_rccl", "collectives_rccl_transport"), ("coll_native", "collectives_rccl_native_transport"),
                      ("rccl_native", "rccl_native_allreduce_f32"), ("c3_variants", "c3_c4_engine_variants"),
                      ("multi_host", "host_path_multi_gpu")):
        if kids[key]:
            out[name] = kids[key]
    return out


def traffic_from_profiles(kernel_substr="k_combine_dram<3, float, float, 64, true, false>"):
    """Per-launch HBM bytes of the default fp32 SUM kernel from the newest
    committed rocprofv3 PMC collection (profiles/<round>/pmc_*counter_collection.csv,
    FETCH_SIZE and WRITE_SIZE collected in separate passes)."""
    import csv
    dirs = sorted({os.path.dirname(p) for p in
                   glob.glob(os.path.join(REPO, "profiles", "*", "pmc_*counter_collection.csv"))})
    best = None
    for d in dirs:
        vals = {"FETCH_SIZE": [], "WRITE_SIZE": []}
        for path in glob.glob(os.path.join(d, "pmc_*counter_collection.csv")):
            with open(path, newline="") as f:
                for row in csv.DictReader(f):
                    if kernel_substr in row["Kernel_Name"] and row["Counter_Name"] in vals:
                        vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
        if vals["FETCH_SIZE"] and vals["WRITE_SIZE"]:
            f_kb = sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"])
            w_kb = sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"])
            # gfx950: FETCH_SIZE reports 1/2 of a 16-B/lane streaming read
            # (MI355X_MICROARCH.md §HBM); both counters are in KiB
            best = (2.0 * f_kb + w_kb) * 1024.0
    return best


def pmc_raw(kernel_substr):
    """Uncorrected per-launch FETCH_SIZE / WRITE_SIZE (KiB) of a kernel from the
    newest committed PMC collection.  Only 16-B-per-lane streaming reads have a
    known gfx950 correction (FETCH_SIZE x 2, MI355X_MICROARCH.md §HBM); other
    widths are reported raw, for ratios between layouts."""
    import csv
    dirs = sorted({os.path.dirname(p) for p in
                   glob.glob(os.path.join(REPO, "profiles", "*", "pmc_*counter_collection.csv"))})
    out = None
    for d in dirs:
        vals = {"FETCH_SIZE": [], "WRITE_SIZE": []}
        for path in glob.glob(os.path.join(d, "pmc_*counter_collection.csv")):
            with open(path, newline="") as f:
                for row in csv.DictReader(f):
                    if kernel_substr in row["Kernel_Name"] and row["Counter_Name"] in vals:
                        vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
        if vals["FETCH_SIZE"] and vals["WRITE_SIZE"]:
            out = {k: round(sum(v) / len(v), 1) for k, v in vals.items()}
    return out


def host_cpu_info():
    """CPU model, sockets, NUMA nodes and the cores this job may use
    (recorded next to the CPU baseline)."""
    info = {"nproc": os.cpu_count()}
    try:
        info["cores_allowed"] = len(os.sched_getaffinity(0))
    except AttributeError:
        pass
    try:
        models, sockets = set(), set()
        with open("/proc/cpuinfo") as f:
            for line in f:
                k, _, v = line.partition(":")
                if k.strip() == "model name":
                    models.add(v.strip())
                elif k.strip() == "physical id":
                    sockets.add(v.strip())
        info["model"] = " / ".join(sorted(models)) or None
        info["sockets"] = len(sockets) or None
    except OSError:
        pass
    info["numa_nodes"] = len(glob.glob("/sys/devices/system/node/node[0-9]*")) or None
    # the cgroup's CPU-time quota (cgroup v2 cpu.max "quota period"): cores'
    # worth of CPU time the job may burn, whatever its affinity mask allows
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        info["cpu_quota_cores"] = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return info


def _median_rate(fn, bytes_per_call, seconds, min_iters=20, warmup=3):
    """3 warm-up calls, then at least `min_iters` timed calls
    (and at least `seconds` of them); returns (median seconds per call, calls)."""
    for _ in range(warmup):
        fn()
    ts, t_end = [], time.perf_counter() + seconds
    while len(ts) < min_iters or time.perf_counter() < t_end:
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2], len(ts)


def cpu_baseline(seconds, elems):
    """The oracle's Op<float>::Sum (the C restatement of op.cpp:42-52) on this
    box's host: one thread (what one MS-MPI rank runs) and every core allotted
    to the job (elements sharded), median of >= 20 calls after 3 warm-ups over
    the full 2 x 256 MiB operands (>> LLC)."""
    import numpy as np
    import oracle
    import msx
    C = msx.C
    n = elems
    rng = np.random.default_rng(0x5EED)
    a = rng.uniform(-1, 1, n).astype(np.float32)
    b = rng.uniform(-1, 1, n).astype(np.float32)
    t1, k1 = _median_rate(lambda: oracle.reduce_local(C.MPI_SUM, C.MPI_FLOAT, a, b), n * BYTES_PER_ELEM, seconds)
    cpu = host_cpu_info()
    out = {"value": round(n * BYTES_PER_ELEM / t1 / 2**30, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
           "sample": f"median of {k1} calls (after 3 warm-ups) of oracle Op<float>::Sum over 2 x {n * 4 >> 20} MiB "
                     f"host buffers, 1 thread = one MS-MPI rank",
           "payload_GiB_s": round(n * 4 / t1 / 2**30, 3), "ms_per_call": round(t1 * 1e3, 3), "cpu": cpu}
    # every host core this job may use (its affinity mask,
    # `cores_allowed`), elements sharded across threads; beside it the rate by
    # thread count, which shows where the host's memory bandwidth (or the
    # job's cgroup CPU quota, `cpu_quota_cores`) stops adding threads paying.
    allowed = max(1, cpu.get("cores_allowed") or os.cpu_count() or 1)
    curve = {}
    for t in sorted({2, 4, 8, 16, 32, 64, 128, allowed}):
        if t > allowed:
            continue
        tt, _ = _median_rate(lambda: oracle.reduce_local(C.MPI_SUM, C.MPI_FLOAT, a, b, nthreads=t),
                             n * BYTES_PER_ELEM, 0.3, min_iters=5, warmup=2)
        curve[str(t)] = round(n * BYTES_PER_ELEM / tt / 2**30, 3)
    if curve:
        out["threads_curve_GiB_s"] = curve
    best = int(max(curve, key=curve.get)) if curve else 1
    if allowed > 1:
        tN, kN = _median_rate(lambda: oracle.reduce_local(C.MPI_SUM, C.MPI_FLOAT, a, b, nthreads=allowed),
                              n * BYTES_PER_ELEM, seconds / 3)
        out["all_cores"] = {"value": round(n * BYTES_PER_ELEM / tN / 2**30, 3), "unit": "GiB/s", "cores": allowed,
                            "payload_GiB_s": round(n * 4 / tN / 2**30, 3), "ms_per_call": round(tN * 1e3, 3),
                            "sample": f"median of {kN} calls after 3 warm-ups, {allowed} threads "
                                      f"(every core of the affinity mask)",
                            "best_threads": best, "best_value": curve.get(str(best))}
    # the same loop by operand size (the host-operand crossover table beside
    # host_path.pageable_by_size_fp32_sum); one thread and the best thread
    # count of the curve
    cores = best
    by = {}
    for nb in HOST_SIZES:
        m = max(1, nb // 4)
        x, y = a[:m].copy(), b[:m].copy()
        t1, _ = _median_rate(lambda: oracle.reduce_local(C.MPI_SUM, C.MPI_FLOAT, x, y), 0, 0.2)
        row = {"us_1core": round(t1 * 1e6, 3)}
        if cores > 1 and nb >= (1 << 20):
            tN, _ = _median_rate(lambda: oracle.reduce_local(C.MPI_SUM, C.MPI_FLOAT, x, y, nthreads=cores), 0, 0.2)
            row[f"us_{cores}cores"] = round(tN * 1e6, 3)
        by[str(nb)] = row
    out["by_size_fp32_sum"] = by
    return out


# Per-(op, type) roofline at the same 256 MiB per operand (reported beside
# `value`, never part of it): the ops of configs 4 and 5 (MAX over DOUBLE,
# BAND over UINT64_T) plus one representative of every kernel family
# (integer wrap, complex arithmetic, logical, loc structs).
PER_OP = [
    ("MPI_SUM", "MPI_FLOAT"), ("MPI_SUM", "MPI_DOUBLE"), ("MPI_SUM", "MPI_INT"),
    ("MPI_SUM", "MPI_INT8_T"), ("MPI_SUM", "MPI_INT64_T"), ("MPI_PROD", "MPI_FLOAT"),
    ("MPI_PROD", "MPI_INT16_T"), ("MPI_SUM", "MPI_C_FLOAT_COMPLEX"),
    ("MPI_PROD", "MPI_C_DOUBLE_COMPLEX"), ("MPI_MAX", "MPI_DOUBLE"), ("MPI_MIN", "MPI_FLOAT"),
    ("MPI_MAX", "MPI_UNSIGNED_CHAR"), ("MPI_BAND", "MPI_UINT64_T"), ("MPI_BXOR", "MPI_BYTE"),
    ("MPI_LAND", "MPI_INT"), ("MPI_LXOR", "MPI_C_BOOL"), ("MPI_MAXLOC", "MPI_2INT"),
    ("MPI_MINLOC", "MPI_DOUBLE_INT"), ("MPI_MAXLOC", "MPI_SHORT_INT"), ("MPI_MINLOC", "MPI_2DOUBLE_PRECISION"),
]


def _mem_available():
    try:
        with open("/proc/meminfo") as f:
            for line in f:
                if line.startswith("MemAvailable:"):
                    return int(line.split()[1]) * 1024
    except OSError:
        pass
    return 16 << 30


def cpu_baseline_collectives(p=8, reps=20, warmup=3):
    """The reference's collective schedules on the host CPU with p THREADS as
    the p ranks (oracle/msx_oracle_threads.c, restated from mpid/reduce.cpp:
    Rabenseifner allreduce :3927-4066, recursive-halving reduce_scatter
    :917-1219 -- the branch c4's wrapped 32-bit byte count selects), each
    thread running its own rank's step loop with memcpy from the peer's buffer
    as the transport and oracle_reduce_local as MPID_Uop_call: what a p-rank
    MS-MPI job on one host computes, SURVEY.md §8(d).  At the configs' own
    per-rank sizes (c3 1 GiB fp32 SUM, c4 4 GiB MAX fp64 send buffer, c5
    512 MiB BAND u64) unless host memory is short, then halved until the
    footprint (send + recv + tmp per rank) fits half of MemAvailable; the
    median of `reps` calls after `warmup` untimed ones (>= 20
    after 3; inputs refilled outside the timed region),
    checked against the closed form.  busBW uses the GPU formulas
    (S/t*2(p-1)/p for allreduce, S/t*(p-1)/p for reduce_scatter)."""
    import oracle
    import msx
    C = msx.C
    avail = _mem_available()
    out = {"ranks": p, "threads": p, "cores": p, "kind": "port",
           "transport": "one memcpy per MPIC_Sendrecv (the reference's shared-memory channel copies twice)",
           "mem_available_GiB": round(avail / 2**30, 1)}
    cfgs = (("c3_allreduce_sum_f32", 0, C.MPI_SUM, C.MPI_FLOAT, 4, 1 << 28, 3.0, 2.0),
            ("c4_reduce_scatter_max_f64", 1, C.MPI_MAX, C.MPI_DOUBLE, 8, (4 << 30) // 8 // p, 2.5, 1.0),
            ("c5_allreduce_band_u64", 0, C.MPI_BAND, C.MPI_UINT64_T, 8, 1 << 26, 3.0, 2.0))
    for name, which, op, dt, esz, count, foot, bus in cfgs:
        full = count
        per_rank_vec = count * (p if which == 1 else 1) * esz          # S: the rank's input bytes
        while count > 1024 and p * foot * (count * (p if which == 1 else 1) * esz) > avail / 2:
            count //= 2
        rc, ts = oracle.coll_threads(which, op, dt, p, count, reps + warmup)
        ts = sorted(ts[warmup:])
        t = ts[len(ts) // 2]
        S = count * (p if which == 1 else 1) * esz
        out[name] = {"bytes_per_rank": S, "config_bytes_per_rank": per_rank_vec,
                     "scaled": count != full, "seconds": round(t, 5), "calls": reps, "warmup_calls": warmup,
                     "correct": rc == 0,
                     "busbw_GB_s": round(S / t / 1e9 * bus * (p - 1) / p, 3)}
        if rc:
            out[name]["rc"] = rc
    return out


def per_op_roofline(L, C, torch, dev, stream, nbytes):
    """GB/s of HBM traffic (2 reads + 1 write per element) per (op, type), from
    HIP events on the launch stream around 10 launches (median of 3 rounds).
    Operands are random bytes interpreted as the MPI type, except floating
    types, which get finite uniform values (no NaN slow path)."""
    import ctypes
    sp = ctypes.c_void_p(stream.cuda_stream)
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    out = {}
    for opn, dtn in PER_OP:
        op, dt = getattr(C, opn), getattr(C, dtn)
        # element stride (pair types: the padded struct, e.g. 16 B for
        # MPI_DOUBLE_INT), not MPI_Type_size's data bytes (12 B)
        sz = ctypes.c_int(L.msx_type_size(dt))
        n = nbytes // sz.value
        assert sz.value > 0 and n * sz.value <= nbytes
        with torch.cuda.stream(stream):
            a.random_(0, 256)
            b.random_(0, 256)
            if dtn in ("MPI_FLOAT", "MPI_C_FLOAT_COMPLEX"):
                a.view(torch.float32).uniform_(-1, 1)
                b.view(torch.float32).uniform_(-1, 1)
            elif dtn in ("MPI_DOUBLE", "MPI_C_DOUBLE_COMPLEX", "MPI_2DOUBLE_PRECISION"):
                a.view(torch.float64).uniform_(-1, 1)
                b.view(torch.float64).uniform_(-1, 1)
            elif dtn == "MPI_DOUBLE_INT":                      # {f64, i32, pad}
                a.view(torch.float64)[0::2].uniform_(-1, 1)
                b.view(torch.float64)[0::2].uniform_(-1, 1)
        ts = []
        for _ in range(3):
            for _ in range(2):
                L.msx_reduce_local_dev(a.data_ptr(), b.data_ptr(), n, dt, op, sp)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(10):
                rc = L.msx_reduce_local_dev(a.data_ptr(), b.data_ptr(), n, dt, op, sp)
                if rc:
                    raise RuntimeError(f"{opn}/{dtn}: rc={rc}")
            e1.record(stream)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 10)
        ms = sorted(ts)[1]
        gbs = 3 * n * sz.value / ms / 1e6
        out[f"{opn}/{dtn}"] = {"us": round(ms * 1e3, 1), "GB_s": round(gbs, 1),
                               "frac": round(gbs / HBM_PEAK_GBS, 4)}
    # mutually misaligned operands (k_combine_shift): `in` a few bytes past
    # 16-byte alignment, `inout` aligned, same 256 MiB
    for dtn, off in (("MPI_FLOAT", 4), ("MPI_INT8_T", 1)):
        dt = getattr(C, dtn)
        esz = L.msx_type_size(dt)
        n = (nbytes - 16) // esz
        ts = []
        for _ in range(3):
            L.msx_reduce_local_dev(a.data_ptr() + off, b.data_ptr(), n, dt, C.MPI_SUM, sp)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(10):
                rc = L.msx_reduce_local_dev(a.data_ptr() + off, b.data_ptr(), n, dt, C.MPI_SUM, sp)
                if rc:
                    raise RuntimeError(f"misaligned {dtn}: rc={rc}")
            e1.record(stream)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 10)
        ms = sorted(ts)[1]
        gbs = 3 * n * esz / ms / 1e6
        out[f"MPI_SUM/{dtn}/in+{off}B"] = {"us": round(ms * 1e3, 1), "GB_s": round(gbs, 1),
                                           "frac": round(gbs / HBM_PEAK_GBS, 4)}
    # the collective combine (k_tree): p = 8 contributions of 32 MiB reduced in
    # the reference's tree order into one output, (p + 1) x 32 MiB of traffic.
    # Sources placed as the engine's window lays out its IN sub-slots (32 MiB
    # + 68 KiB apart, msx_transport.cpp sub_skew); "tree8_pow2_stride" is the
    # same call with the sources exactly 32 MiB apart.
    p, m = 8, nbytes // 8 // 4
    skew = 68 << 10
    del a
    a = torch.empty(p * (m * 4 + skew), dtype=torch.uint8, device=dev)
    a.view(torch.float32).uniform_(-1, 1)
    srcs = (ctypes.c_void_p * p)(*[a.data_ptr() + r * (m * 4 + skew) for r in range(p)])
    srcs_pow2 = (ctypes.c_void_p * p)(*[a.data_ptr() + r * m * 4 for r in range(p)])

    def time_tree(srcs=srcs):
        ts = []
        for _ in range(3):
            L.msx_reduce_tree_dev(srcs, p, b.data_ptr(), m, C.MPI_FLOAT, C.MPI_SUM, sp)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(10):
                rc = L.msx_reduce_tree_dev(srcs, p, b.data_ptr(), m, C.MPI_FLOAT, C.MPI_SUM, sp)
                if rc:
                    raise RuntimeError(f"tree: rc={rc}")
            e1.record(stream)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 10)
        return sorted(ts)[1]

    def entry(ms):
        gbs = (p + 1) * m * 4 / ms / 1e6
        return {"us": round(ms * 1e3, 1), "GB_s": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}

    out["tree8/MPI_SUM/MPI_FLOAT"] = entry(time_tree())
    # HBM bytes per launch from the committed PMC passes (16-B streaming loads:
    # FETCH_SIZE doubled per the gfx950 calibration), against (p + 1) * 32 MiB
    raw = pmc_raw("k_tree<3, float, float, 256, false, 8, 1, false, false>")
    if raw:
        out["tree8/MPI_SUM/MPI_FLOAT"].update(
            {"pmc_raw_kib": raw, "traffic": int((2 * raw["FETCH_SIZE"] + raw["WRITE_SIZE"]) * 1024),
             "bytes_per_launch": (p + 1) * m * 4})
    out["tree8_pow2_stride/MPI_SUM/MPI_FLOAT"] = entry(time_tree(srcs_pow2))
    del a, b
    return out


# rocprofv3 kernel symbol of each pack-table entry (for the PMC traffic lookup)
KERNEL_OF = {
    "vector_16B_blocks_stride32B": {"pack": "k_dt_pack<16, true, true, false>",
                                    "unpack": "k_dt_pack<16, true, true, true>"},
    "double_int_records_12of16B": {"pack": "k_dt_pack<4, true, true, false>",
                                   "unpack": "k_dt_pack<4, true, true, true>"},
    "subarray3d_fp32_rows1536B": {"pack": "k_dt_pack_tile<16, true, true, false>",
                                  "unpack": "k_dt_pack_tile<16, true, true, true>"},
}


def pack_roofline(L, C, torch, dev, stream):
    """MPI_Pack / MPI_Unpack kernels (msx_pack.hip) through msx_pack_dev /
    msx_unpack_dev on device buffers: algorithmic HBM bytes = 2 x packed size
    per call (each packed byte read once and written once), timed with HIP
    events on the launch stream (median of 3 rounds of 10 calls).  Layouts:
    a 16-B-block vector (regular map, 16-B granules), MPI_DOUBLE_INT records
    (12 of every 16 B, 4-B granules) and a 3-D fp32 subarray (irregular run
    list, binary-search map).  Every layout is checked against torch first."""
    import ctypes
    sp = ctypes.c_void_p(stream.cuda_stream)
    out = {}

    def mk(fn, *a):
        t = ctypes.c_int()
        assert fn(*a, ctypes.byref(t)) == 0, msx_err()
        assert L.MPI_Type_commit(ctypes.byref(t)) == 0
        return t

    def msx_err():
        import msx
        return msx.last_error()

    ia = lambda v: (ctypes.c_int * len(v))(*v)
    nf = 1 << 26                                           # 256 MiB of fp32 typed data
    typed = torch.randn(nf, device=dev)
    layouts = []
    t = mk(L.MPI_Type_vector, nf // 8, 4, 8, C.MPI_FLOAT)
    layouts.append(("vector_16B_blocks_stride32B", t, 1, typed.view(-1, 8)[:, :4].contiguous()))
    n_di = nf // 4                                          # 16 B records
    layouts.append(("double_int_records_12of16B", ctypes.c_int(C.MPI_DOUBLE_INT), n_di,
                    typed.view(-1, 4)[:, :3].contiguous()))
    dims, sub, st = (256, 512, 512), (192, 400, 384), (32, 56, 64)
    t3 = mk(L.MPI_Type_create_subarray, 3, ia(dims), ia(sub), ia(st), C.MPI_ORDER_C, C.MPI_FLOAT)
    v3 = typed.view(*dims)[st[0]:st[0] + sub[0], st[1]:st[1] + sub[1], st[2]:st[2] + sub[2]].contiguous()
    layouts.append(("subarray3d_fp32_rows1536B", t3, 1, v3))
    for name, t, count, want in layouts:
        packed = torch.empty(want.numel() * want.element_size(), dtype=torch.uint8, device=dev)
        nb = packed.numel()
        rc = L.msx_pack_dev(typed.data_ptr(), count, t.value, packed.data_ptr(), sp)
        torch.cuda.synchronize()
        if rc or not torch.equal(packed, want.view(-1).view(torch.uint8)):
            raise RuntimeError(f"pack parity failed for {name}: rc={rc}")
        # HBM moves whole 32-B sectors: a gapped typed side touches more bytes
        # than it carries (round 4: a bare 16-of-32-B store kernel, the probe
        # library's gapped-store mode, reports WRITE_SIZE = 2x its data too), so each entry also reports
        # packed bytes + the typed side's touched 32-B sectors
        typed_sectors = {"vector_16B_blocks_stride32B": 2 * nb, "double_int_records_12of16B": nb * 16 // 12,
                         "subarray3d_fp32_rows1536B": nb}[name]
        res = {"packed_bytes": nb, "algorithmic_bytes_per_call": 2 * nb,
               "touched_sector_bytes_per_call": nb + typed_sectors}
        for label, fn, a, b in (("pack", L.msx_pack_dev, typed, packed), ("unpack", L.msx_unpack_dev, packed, typed)):
            ts = []
            for _ in range(3):
                fn(a.data_ptr(), count, t.value, b.data_ptr(), sp)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(10):
                    fn(a.data_ptr(), count, t.value, b.data_ptr(), sp)
                e1.record(stream)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / 10)
            ms = sorted(ts)[1]
            gbs = 2 * nb / ms / 1e6
            sec = res["touched_sector_bytes_per_call"] / ms / 1e6
            res[label] = {"us": round(ms * 1e3, 1), "GB_s": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
                          "sector_GB_s": round(sec, 1), "frac_sector": round(sec / HBM_PEAK_GBS, 4),
                          "kernel": KERNEL_OF[name][label]}
            res[label]["pmc_raw_kib"] = pmc_raw(KERNEL_OF[name][label])
        out[name] = res
        del packed
    for t in (layouts[0][1], t3):
        L.MPI_Type_free(ctypes.byref(t))
    del typed
    return out


def cold_cache_launch(P, torch, dev, stream, src, acc, n, reps=12, mixes=True):
    """The headline launch with the Infinity Cache cold.  MI355X has a 256 MiB
    memory-side cache (MALL); back to back on the same 256 MiB operands it
    serves part of every launch (round 3: 256 MiB 115 us warm vs 140 us cold;
    from 512 MiB per operand on, warm = cold).  Here each launch follows a
    read + write pass over 1 GiB of other data and is timed alone with HIP
    events; the DRAM-only rate next to the 2R+1W ceiling the same cold method
    gives the copy-like stream mix is what the kernel does without the cache.
    The launches run the default kernel body (k_combine_dram's) under the probe
    library's symbol k_probe_combine<1, 64, true, false, 128>, so these single
    launches stay out of the headline symbol's rocprof average.  Reported
    beside `value`, never part of it."""
    from msx import probe
    sp = ctypes.c_void_p(stream.cuda_stream)
    v = probe.variants().get("default_body_probe")
    if v is None:
        return {"error": "default_body_probe variant missing"}

    def step():
        if P.msxp_variant_run(v, src.data_ptr(), acc.data_ptr(), n, sp):
            raise RuntimeError("probe variant launch failed")
    flush = torch.empty(1 << 30, dtype=torch.uint8, device=dev)

    def flush_cache():
        P.msxp_hbm(probe.READ1, flush.data_ptr(), flush.data_ptr(), flush.numel(), sp)
        P.msxp_hbm(probe.WRITE1, flush.data_ptr(), flush.data_ptr(), flush.numel(), sp)
    ts, warm = [], []
    for _ in range(reps):
        flush_cache()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        step()
        e1.record(stream)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        step()
        e1.record(stream)
        torch.cuda.synchronize()
        warm.append(e0.elapsed_time(e1))
    # the same cold method for the copy (1R1W) and two-read stream mixes of the
    # HBM probe, on scratch operands of the same size
    a2 = torch.empty(n * 4, dtype=torch.uint8, device=dev)
    b2 = torch.empty(n * 4, dtype=torch.uint8, device=dev)
    a2.random_(0, 256)
    b2.random_(0, 256)
    torch.cuda.synchronize()
    kinds, mixes = (((probe.COPY, "copy_r1w1", 2), (probe.COPY_DISPATCH_ORDER, "copy_r1w1_dispatch_order", 2),
                     (probe.COPY_XCD_RUNS, "copy_r1w1_xcd_runs128", 2), (probe.READ2, "read2", 2))
                    if mixes else ()), {}
    for mode, name, streams in kinds:
        pt = []
        for _ in range(reps):
            flush_cache()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            P.msxp_hbm(mode, a2.data_ptr(), b2.data_ptr(), n * 4, sp)
            e1.record(stream)
            torch.cuda.synchronize()
            pt.append(e0.elapsed_time(e1))
        pms = sorted(pt)[reps // 2]
        mixes[name] = round(streams * n * 4 / pms / 1e6, 1)
    del flush, a2, b2
    cms, wms = sorted(ts)[reps // 2], sorted(warm)[reps // 2]
    gbs = n * BYTES_PER_ELEM / cms / 1e6
    return {"cold_us": round(cms * 1e3, 1), "cold_GB_s": round(gbs, 1), "cold_frac": round(gbs / HBM_PEAK_GBS, 4),
            "warm_single_us": round(wms * 1e3, 1), "cold_probe_GB_s": mixes,
            "method": "median of 12 single launches, each after a 1 GiB read + write pass over other data "
                      "(cold) or right after the previous launch (warm); HIP events on the launch stream; "
                      "the default kernel body under the probe symbol k_probe_combine<1, 64, true, false, 128>"}


def hbm_ceiling_probe(P, torch, dev, stream, nbytes):
    """What this GPU's HBM delivers for other stream mixes on the same
    2 x 256 MiB operands, in the tile geometry (k_probe: 16 B per lane,
    256-lane workgroups, one tile each, XCD-contiguous, non-temporal loads):
    2 reads, 1 read, 1 write, 1 read + 1 write; and the copy in the combine's
    default geometry at this size (k_copy_dram: one-wave workgroups in
    dispatch order).  Median of 3 rounds of 10 launches, HIP events on the
    launch stream.  Context for the roofline's `frac` (which stays against
    the 8 TB/s spec peak).  Bench-only kernels (libmsx_probe.so)."""
    sp = ctypes.c_void_p(stream.cuda_stream)
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    with torch.cuda.stream(stream):
        a.random_(0, 256)
        b.random_(0, 256)
    out = {}
    for mode, name, streams in ((0, "read2", 2), (3, "read1", 1), (1, "write1", 1), (2, "copy_r1w1", 2),
                                (9, "copy_r1w1_dispatch_order", 2), (10, "copy_r1w1_xcd_runs128", 2),
                                (6, "write_16of32B", 0.5), (7, "read_16of32B", 0.5)):
        ts = []
        for _ in range(3):
            for _ in range(2):
                P.msxp_hbm(mode, a.data_ptr(), b.data_ptr(), nbytes, sp)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(10):
                rc = P.msxp_hbm(mode, a.data_ptr(), b.data_ptr(), nbytes, sp)
                if rc:
                    raise RuntimeError(f"probe {name}: rc={rc}")
            e1.record(stream)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 10)
        ms = sorted(ts)[1]
        gbs = streams * nbytes / ms / 1e6
        out[name] = {"us": round(ms * 1e3, 1), "GB_s": round(gbs, 1), "frac_of_spec": round(gbs / HBM_PEAK_GBS, 4)}
    del a, b
    return out


def rma_self_roofline(L, C, torch, dev, n):
    """One-sided MPI_Accumulate (MPI_SUM, fp32) into this rank's own device
    window: the reference applies a self-targeted accumulate at the call
    (win.cpp:1570-1590, MPIDI_Win_local_accumulate), here through the combine
    kernels.  Wall clock per blocking call (launch + sync included), 12 B per
    element of HBM traffic like the local combine."""
    import ctypes
    win_buf = torch.zeros(n, device=dev)
    origin = torch.rand(n, device=dev)
    torch.cuda.synchronize()
    win = ctypes.c_int()
    if L.MPI_Win_create(win_buf.data_ptr(), n * 4, 4, C.MPI_INFO_NULL, C.MPI_COMM_WORLD, ctypes.byref(win)):
        return {"error": "MPI_Win_create failed"}
    acc = lambda: L.MPI_Accumulate(origin.data_ptr(), n, C.MPI_FLOAT, 0, 0, n, C.MPI_FLOAT, C.MPI_SUM, win)
    for _ in range(3):
        acc()
    reps, t0 = 20, time.perf_counter()
    for _ in range(reps):
        rc = acc()
        if rc:
            break
    dt = (time.perf_counter() - t0) / reps
    correct = None
    if not rc:
        # 23 accumulations of the same origin into zeros: exact check on a sample
        ref = torch.zeros(4096, device=dev)
        for _ in range(23):
            ref += origin[:4096]
        correct = bool(torch.equal(win_buf[:4096], ref))
    L.MPI_Win_free(ctypes.byref(win))
    gbs = 12 * n / dt / 1e9
    return {"bytes_per_call": 12 * n, "ms_per_call": round(dt * 1e3, 3), "GB_s": round(gbs, 1),
            "frac": round(gbs / HBM_PEAK_GBS, 4), "correct": correct}


def launch_ranks(args):
    """`bench.py --gpus N` without a launcher: start N rank processes of this
    script (one per GPU: LOCAL_RANK = rank; on a box with fewer GPUs they share
    them round-robin), the way `torch.distributed.run --nproc-per-node N` would,
    before this process touches any GPU.  Rank 0 prints the JSON line; the exit
    status is the first failing rank's.  A rank that fails takes the others
    down after a grace period, so nothing waits for gloo's 30-minute timeout."""
    import signal
    import socket
    import subprocess
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(args.gpus),
                    "LOCAL_WORLD_SIZE": str(args.gpus), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      start_new_session=True))
    rc, failed_at = 0, None
    while any(pr.poll() is None for pr in procs):
        bad = [pr for pr in procs if pr.poll() not in (None, 0)]
        if bad and failed_at is None:
            failed_at = time.time()
            rc = bad[0].returncode
        if failed_at is not None and time.time() - failed_at > 60:
            for pr in procs:
                if pr.poll() is None:
                    os.killpg(pr.pid, signal.SIGKILL)
        time.sleep(0.2)
    for pr in procs:
        if pr.returncode and not rc:
            rc = pr.returncode
    return rc


def main():
    args = parse()
    if args.rccl_native_child:
        rccl_native_child_main(args.rccl_native_child, args.coll_scale)
        return
    if args.multi_host_child:
        multi_host_child_main(args.multi_host_child, args.elems)
        return
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args))
    if env_world is not None and int(env_world) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}: the launcher and the flag disagree")
    import torch
    import torch.distributed as dist
    import msx

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        with stdout_to_stderr():
            dist.init_process_group("gloo", init_method="env://")
    # one rank per GPU; ranks beyond the visible GPUs share them round-robin
    # (lets the N>1 path run on a one-GPU box too)
    local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    # the library is a per-rank singleton here (no collective in the data path)
    os.environ["MSX_SIZE"], os.environ["MSX_RANK"], os.environ["MSX_DEVICE"] = "1", "0", str(local)
    L = msx.init(errors_return=True)
    C = msx.C
    from msx import probe
    P = probe.lib()                          # bench-only measurement kernels

    n = args.elems
    g = torch.Generator(device=dev).manual_seed(0x5EED + rank)
    src = torch.rand(n, device=dev, generator=g) * 2 - 1
    acc = torch.rand(n, device=dev, generator=g) * 2 - 1
    stream = torch.cuda.Stream(dev)          # the launch stream of every timed kernel
    torch.cuda.set_stream(stream)
    sp = ctypes.c_void_p(stream.cuda_stream)

    def step():
        rc = L.msx_reduce_local_dev(src.data_ptr(), acc.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM, sp)
        if rc:
            raise RuntimeError(f"msx_reduce_local_dev: {rc} {msx.last_error()}")

    # correctness of the timed kernel on this exact data (one IEEE add / element)
    ref = acc + src
    step()
    torch.cuda.synchronize()
    if not torch.equal(acc.view(torch.int32), ref.view(torch.int32)):
        raise RuntimeError("parity check failed before timing")
    del ref

    sweep = {}
    if args.sweep and rank == 0:
        # interleaved rounds in one process (cdna_hip_programming.md §5.4 rule
        # 24): the product kernel and the probe library's variants of its body
        runs = {"product": step}
        for name, v in probe.variants().items():
            runs[name] = (lambda v=v: P.msxp_variant_run(v, src.data_ptr(), acc.data_ptr(), n, sp))
        times = {k: [] for k in runs}
        for _ in range(3):
            for key, fn in runs.items():
                for _ in range(3):
                    fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(10):
                    fn()
                e1.record(stream)
                torch.cuda.synchronize()
                times[key].append(e0.elapsed_time(e1) / 10)
        for key, ts in times.items():
            ms = sorted(ts)[len(ts) // 2]
            sweep[key] = round(n * BYTES_PER_ELEM / ms / 1e6, 1)
            print(f"{key}: {ms * 1e3:.1f} us {sweep[key]:.0f} GB/s", file=sys.stderr)
        # operand placement: the default kernel with `in` and `inout` carved
        # from one allocation at exactly 256 MiB apart vs skewed by a few KiB
        # (HBM bank aliasing of two streams a power of two apart)
        pool = torch.empty(2 * n * 4 + (2 << 20), dtype=torch.uint8, device=dev)
        pool.view(torch.float32)[: (pool.numel() // 4)].uniform_(-1, 1)
        atimes = {}
        for _ in range(3):
            for sk in (0, 4 << 10, 68 << 10, (1 << 20) + (68 << 10)):
                pa, pb = pool.data_ptr(), pool.data_ptr() + n * 4 + sk
                for _ in range(3):
                    L.msx_reduce_local_dev(pa, pb, n, C.MPI_FLOAT, C.MPI_SUM, sp)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(10):
                    L.msx_reduce_local_dev(pa, pb, n, C.MPI_FLOAT, C.MPI_SUM, sp)
                e1.record(stream)
                torch.cuda.synchronize()
                atimes.setdefault(sk, []).append(e0.elapsed_time(e1) / 10)
        for sk, ts in atimes.items():
            ms = sorted(ts)[1]
            sweep[f"operand_gap_256MiB_plus_{sk}"] = round(n * BYTES_PER_ELEM / ms / 1e6, 1)
            print(f"operands 256 MiB + {sk} B apart: {ms * 1e3:.1f} us {sweep[f'operand_gap_256MiB_plus_{sk}']:.0f} GB/s",
                  file=sys.stderr)
        del pool

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    # timed region: K back-to-back launches on `stream`, bracketed by HIP
    # events on that stream (kernel time incl. launch gaps) and by the host
    # clock between barrier + synchronize on both sides (value).  Each rank's
    # clock stops at its own final synchronize, before the closing barrier:
    # the MAX over ranks below covers the slowest rank, and the barrier's own
    # TCP round trips (gloo, ~0.1-1 ms for 8 processes) stay out of a region
    # that lasts ~2 ms at K = 20.
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    kern_ms = ev0.elapsed_time(ev1) / args.steps

    t = torch.tensor([elapsed, kern_ms], dtype=torch.float64)
    kern_all = [kern_ms]
    if world > 1:
        parts = [torch.zeros(2, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(parts, t)
        kern_all = [float(x[1]) for x in parts]
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kern_ms_max = float(t[0]), float(t[1])

    # N > 1: the collective configs in child MPI processes (not part of
    # `value`), under one wall budget (run_children)
    kids = None
    if world > 1 and not args.no_collectives:
        kids = run_children(dist, world, rank, local, args.coll_scale, n, torch.cuda.device_count() >= world,
                            args.no_host_path)
    # host-memory path (the MPI buffers start and end in host memory): measured
    # on rank 0 only, reported beside the device-resident value.
    host = None
    if rank == 0 and world == 1 and not args.no_host_path:
        host = {}
        a_h = src.cpu()
        for label, pin, mode in (("pageable", False, 0), ("pageable_staged", False, 2),
                                 ("pinned_zero_copy", True, 0), ("pinned_staged", True, 1)):
            L.msx_set_host_mode(mode)
            ah = a_h.pin_memory() if pin else a_h.clone()
            bh = acc.cpu()
            bh = bh.pin_memory() if pin else bh
            L.MPI_Reduce_local(ah.data_ptr(), bh.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM)
            reps, t1 = 3, time.perf_counter()
            for _ in range(reps):
                rc = L.MPI_Reduce_local(ah.data_ptr(), bh.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM)
                assert rc == 0, msx.last_error()
            dt_h = (time.perf_counter() - t1) / reps
            host[label] = {"ms_per_call": round(dt_h * 1e3, 2),
                           "payload_GiB_s": round(n * 4 / dt_h / 2**30, 2),
                           "traffic_GiB_s": round(n * BYTES_PER_ELEM / dt_h / 2**30, 2)}
        L.msx_set_host_mode(0)
        # crossover table: pageable host operands by size, the
        # default host path (bounce buffers up to 256 KiB, then pinned for the
        # call); cpu_baseline.by_size times the CPU loop on the same sizes
        import numpy as np
        by = {}
        for nb in HOST_SIZES:
            m = max(1, nb // 4)
            ha = np.random.default_rng(1).uniform(-1, 1, m).astype(np.float32)
            hb = np.random.default_rng(2).uniform(-1, 1, m).astype(np.float32)
            reps = 200 if nb <= (1 << 20) else (20 if nb <= (16 << 20) else 5)
            for _ in range(3):
                L.MPI_Reduce_local(ha.ctypes.data, hb.ctypes.data, m, C.MPI_FLOAT, C.MPI_SUM)
            ts = []
            for _ in range(reps):
                t1 = time.perf_counter()
                rc = L.MPI_Reduce_local(ha.ctypes.data, hb.ctypes.data, m, C.MPI_FLOAT, C.MPI_SUM)
                ts.append(time.perf_counter() - t1)
                assert rc == 0, msx.last_error()
            ts.sort()
            by[str(nb)] = {"us": round(ts[len(ts) // 2] * 1e6, 2),
                           "payload_GiB_s": round(nb / ts[len(ts) // 2] / 2**30, 3)}
        host["pageable_by_size_fp32_sum"] = by
        # blocking MPI_Reduce_local on device buffers (adds launch + sync per call)
        reps, t1 = 10, time.perf_counter()
        for _ in range(reps):
            L.MPI_Reduce_local(src.data_ptr(), acc.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM)
        dt_b = (time.perf_counter() - t1) / reps
        host["device_blocking_MPI_Reduce_local_GiB_s"] = round(n * BYTES_PER_ELEM / dt_b / 2**30, 1)

    per_op = None
    if rank == 0 and world == 1 and not args.no_per_op:
        per_op = per_op_roofline(L, C, torch, dev, stream, n * 4)
    pack = None
    if rank == 0 and world == 1 and not args.no_pack:
        pack = pack_roofline(L, C, torch, dev, stream)
    rma = hbm = cold = None
    if rank == 0 and world == 1 and not args.no_per_op:
        rma = rma_self_roofline(L, C, torch, dev, n)
        hbm = hbm_ceiling_probe(P, torch, dev, stream, n * 4)
    if rank == 0:
        # SURVEY.md §7 "use cold buffers": the headline launch with the Infinity
        # Cache flushed first, reported in `roofline` beside the back-to-back frac
        cold = cold_cache_launch(P, torch, dev, stream, src, acc, n, mixes=(world == 1 and not args.no_per_op))

    if rank == 0:
        total_bytes = world * args.steps * n * BYTES_PER_ELEM
        value = total_bytes / elapsed / 2**30
        achieved = n * BYTES_PER_ELEM / (kern_ms / 1e3) / 1e9      # GB/s, rank 0's kernel
        traffic = traffic_from_profiles()
        out = {
            "metric": "GiB/s device-resident MPI_SUM local-reduce fp32 (HBM traffic, 12 B/element)",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic uniform[-1,1) fp32, seeded per rank, resident in HBM",
            "config": {"workload": "MPI_SUM MPI_FLOAT local-reduce, 256 MiB per operand per GPU "
                                   "(BASELINE.json configs[1])",
                       "elements_per_gpu": n, "bytes_per_operand": n * 4,
                       "parallelism": f"{world} rank(s), one per GPU, independent shards"},
            "payload_GiB_s": round(world * args.steps * n * 4 / elapsed / 2**30, 2),
            "pct_hbm_peak": round(100 * value * 2**30 / 1e9 / (world * HBM_PEAK_GBS), 2),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": (round(traffic) if traffic else None),
                         "bytes_per_launch": n * BYTES_PER_ELEM,
                         "kernel_us_mean": round(kern_ms * 1e3, 2),
                         "timing": "HIP events around the K launches on the launch stream / K",
                         "kernel_us_mean_max_rank": round(kern_ms_max * 1e3, 2),
                         "kernel_us_mean_per_rank": [round(k * 1e3, 2) for k in kern_all]},
        }
        if cold is not None and "cold_frac" in cold:
            # the same kernel body with the 256 MiB Infinity Cache flushed before
            # each launch: the DRAM-only fraction (the >= 70 % target is against it)
            out["roofline"].update({"frac_cold": cold["cold_frac"], "achieved_cold": cold["cold_GB_s"],
                                    "kernel_us_cold": cold["cold_us"],
                                    "cold_method": "median of 12 single launches, each after a 1 GiB read + "
                                                   "write pass over other data (flushes the 256 MiB MALL); "
                                                   "the default body (k_combine_dram's) under the bench-only "
                                                   "symbol k_probe_combine<1, 64, true, false, 128>"})
        if host is not None:
            out["host_path"] = host
        if kids is not None:
            out.update(collectives_report(kids))
        if per_op is not None:
            out["per_op_roofline_hbm"] = per_op
        if pack is not None:
            out["datatype_pack_roofline_hbm"] = pack
        if rma is not None:
            out["rma_self_accumulate_f32"] = rma
        if hbm is not None:
            out["hbm_ceiling_probe"] = hbm
        if cold is not None:
            out["infinity_cache"] = cold
        if sweep:
            out["variant_sweep_GB_s"] = sweep
        if world == 1:
            del src, acc
            torch.cuda.empty_cache()
            out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, n)
            hp = out.get("host_path", {}).get("pageable_by_size_fp32_sum")
            cb = out["cpu_baseline"].get("by_size_fp32_sum")
            if hp and cb:
                # the smallest pageable host operand size at which the offload beats
                # one core running the reference loop (INTEGRATION.md §2 routes
                # host operands of the op table to that loop)
                sizes = sorted(int(k) for k in hp if str(k) in cb)
                wins = [b for b in sizes if hp[str(b)]["us"] < cb[str(b)]["us_1core"]]
                out["host_path"]["crossover"] = {
                    "bytes_offload_beats_1core": wins[0] if wins else None,
                    "per_size_us_offload_vs_1core": {str(b): [hp[str(b)]["us"], cb[str(b)]["us_1core"]]
                                                     for b in sizes}}
            if not args.no_collectives:
                out["cpu_baseline_collectives"] = cpu_baseline_collectives(8)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
