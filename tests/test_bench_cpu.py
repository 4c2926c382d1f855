"""CPU: bench.py's launcher contract (no GPU needed for these paths)."""
import os
import subprocess
import sys

import msx

REPO = msx.REPO_ROOT


def test_gpus_flag_must_match_the_launcher_world_size():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    pr = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4"], env=env,
                        capture_output=True, text=True, timeout=60)
    assert pr.returncode != 0
    assert "WORLD_SIZE=2" in pr.stderr and "--gpus 4" in pr.stderr
    assert pr.stdout == ""


def test_cpu_info_and_median_helpers():
    sys.path.insert(0, REPO)
    import bench
    info = bench.host_cpu_info()
    assert info["nproc"] >= 1 and "model" in info and "numa_nodes" in info
    calls = []
    t, k = bench._median_rate(lambda: calls.append(1), 0, 0.0)
    assert k == 20 and len(calls) == 23 and t >= 0          # 3 warm-ups + 20 timed


def test_threaded_collective_baseline_is_correct():
    """oracle/msx_oracle_threads.c (bench.py cpu_baseline_collectives): p
    threads as ranks run the reference's Rabenseifner allreduce / recursive-
    halving reduce_scatter_block step loops; ragged counts (count % p != 0) and
    p = 2, 4, 8 must give the closed-form result on every rank."""
    sys.path.insert(0, REPO)
    import oracle
    C = msx.C
    for which, op, dt in ((0, C.MPI_SUM, C.MPI_FLOAT), (0, C.MPI_BAND, C.MPI_UINT64_T),
                          (1, C.MPI_MAX, C.MPI_DOUBLE)):
        for p in (2, 4, 8):
            for count in (p, 1000 + p - 1, (1 << 16) + 3):
                rc, ts = oracle.coll_threads(which, op, dt, p, count, 2)
                assert rc == 0, (which, p, count, rc)
                assert len(ts) == 2 and all(t > 0 for t in ts)
    # refused: non-power-of-two p, unsupported type
    assert oracle.coll_threads(0, C.MPI_SUM, C.MPI_FLOAT, 6, 1000, 1)[0] == C.MPI_ERR_ARG
    assert oracle.coll_threads(0, C.MPI_SUM, C.MPI_INT, 8, 1000, 1)[0] == C.MPI_ERR_ARG


def test_cpu_baseline_collectives_scales_to_memory(monkeypatch):
    """At the configs' sizes when host memory allows, halved otherwise; each
    entry states its size, threads and busBW (VERDICT r03 'Next' 7)."""
    sys.path.insert(0, REPO)
    import bench
    monkeypatch.setattr(bench, "_mem_available", lambda: 3 << 30)   # force scaling on this host
    out = bench.cpu_baseline_collectives(8, reps=1, warmup=1)
    assert out["threads"] == 8 and out["kind"] == "port"
    for k in ("c3_allreduce_sum_f32", "c4_reduce_scatter_max_f64", "c5_allreduce_band_u64"):
        e = out[k]
        assert e["correct"] and e["busbw_GB_s"] > 0 and e["scaled"], e
        assert e["bytes_per_rank"] < e["config_bytes_per_rank"]


def test_wall_budget_bounds_every_hung_child():
    """bench.py N > 1: with EVERY child hanging until its time limit, the
    children end within the wall budget minus the reserve for the JSON line,
    whatever the start-up took (VERDICT r05 'Next' 1)."""
    sys.path.insert(0, REPO)
    import bench
    assert set(bench.CHILD_ORDER) == set(bench.CHILD_CAP_S)
    for startup in (5.0, 60.0, 150.0, 300.0, 400.0):
        el, ran = startup, []
        for name in bench.CHILD_ORDER:
            t = bench.child_timeout(name, el)
            if t is not None:
                assert t >= bench.MIN_CHILD_S
                el += t                        # the child hangs: killed at its limit
                ran.append(name)
        assert el <= max(startup, bench.WALL_BUDGET_S - bench.RESERVE_S) + 1e-9, (startup, el, ran)
        if startup <= 60.0:
            assert ran[0] == "ipc_core"        # the headline configs always get their slot
    # the worst case the driver saw before the budget: ~1,380 s of child limits
    assert sum(bench.CHILD_CAP_S.values()) > bench.WALL_BUDGET_S


_CHILDREN_SCRIPT = r'''
import json, os, sys, time
sys.path.insert(0, os.environ["REPO"])
import torch.distributed as dist
import bench
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", rank=rank, world_size=world)
if os.environ.get("FAKE_LATE"):
    bench.T_START = time.time() - (bench.WALL_BUDGET_S - bench.RESERVE_S - 1)
calls = []
def plane(bw):
    return {"c3_allreduce_sum_f32": {"correct": True, "busbw_GB_s": bw, "seconds": 0.004},
            "c4_reduce_scatter_max_f64": {"correct": True, "busbw_GB_s": bw / 2, "seconds": 0.009},
            "c5_iallreduce_band_u64": {"correct": True, "busbw_GB_s": bw / 4, "seconds": 0.002}}
class Fake:
    @staticmethod
    def collectives(world, rank, local, scale, transport, extra, tag, port_off, parts, timeout):
        calls.append([transport, parts, tag, port_off, timeout])
        if transport == "rccl" and rank == 1:
            return {"error": {"stage": "c3", "text": "fake failure"}}
        if rank != 0:
            return {}
        r = plane({"ipc": 400.0, "rccl": 300.0, "rccl_native": 350.0}[transport])
        if transport == "ipc" and parts == "core":
            r["peer_write_probe"] = {"outbound_GB_s_per_gpu": 500.0}
        return r
    @staticmethod
    def rccl_allreduce(world, rank, local, scale, timeout):
        return {"correct": True, "busbw_GB_s": 450.0} if rank == 0 else {}
    @staticmethod
    def multi_host(n, timeout):
        return {"gpus": 2, "timeout": timeout}
kids = bench.run_children(dist, world, rank, local=rank, scale=1.0, n=2, distinct=True, no_host_path=False,
                          runners=Fake)
if rank == 0:
    print(json.dumps({"report": bench.collectives_report(kids), "calls": calls}))
dist.barrier()
dist.destroy_process_group()
'''


def _run_children(port, **env_extra):
    procs = []
    for r in range(2):
        env = dict(os.environ, REPO=REPO, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), MSX_BENCH_VARIANTS_AT="2", **env_extra)
        procs.append(subprocess.Popen([sys.executable, "-c", _CHILDREN_SCRIPT], env=env, text=True,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE))
    outs = [p.communicate(timeout=120) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e
    import json
    return json.loads(outs[0][0].strip().splitlines()[-1])


def test_children_sequence_and_report_on_distinct_gpus():
    """bench.py N > 1 on distinct GPUs (the driver's one-shot 8-GPU run, which
    no test here can launch): two gloo ranks drive run_children with fake child
    processes; every plane is summarized with its fraction of the measured
    links, a non-zero rank's failure is reported by rank, the variant run and
    the host split take their budgeted turns in CHILD_ORDER."""
    res = _run_children(29611)
    rep, calls = res["report"], res["calls"]
    assert [c[:3] for c in calls] == [["ipc", "core", ""], ["rccl", "core", ""], ["rccl_native", "core", ""],
                                      ["ipc", "c3c4", "_pipeline"], ["ipc", "extras", "_extras"]]
    assert all(c[4] is not None and c[4] >= 20 for c in calls)
    sm = rep["collectives_summary"]
    assert sm["plane"] == "xgmi" and sm["measured_links_GB_s_per_gpu"] == 500.0
    assert sm["ipc"]["c3"]["busbw_frac_measured_links"] == 0.8
    assert sm["ipc"]["c4"]["busbw_frac_measured_links"] == 0.4
    assert sm["rccl_native"]["c5"]["busbw_frac_measured_links"] == 0.175
    assert sm["rccl"]["error"]["rank"] == 1                       # rank 1's failure, by rank
    assert rep["collectives_rccl_transport"]["errors"][0]["text"] == "fake failure"
    assert sm["rccl_own_allreduce_f32"]["busbw_frac_measured_links"] == 0.9
    v = rep["c3_c4_engine_variants"]["pipeline"]
    assert v["c3"]["busbw_GB_s"] == 400.0 and v["env"] == dict(__import__("bench").C3_VARIANTS)["pipeline"]
    steps = [s["name"] for s in rep["wall_budget"]["steps"]]
    assert steps == ["ipc_core", "rccl_core", "rccl_native_core", "rccl_allreduce", "variant_pipeline",
                     "ipc_extras", "multi_host"]
    assert [s["name"] for s in rep["wall_budget"]["steps"] if s.get("error")] == ["rccl_core"]
    assert rep["host_path_multi_gpu"]["gpus"] == 2


def test_children_skipped_when_the_budget_is_spent():
    """Started with the wall budget already spent: every child is skipped (and
    recorded as such), no child process runs, the report still forms."""
    res = _run_children(29613, FAKE_LATE="1")
    rep, calls = res["report"], res["calls"]
    assert calls == []
    assert all(s.get("skipped") == "wall budget" for s in rep["wall_budget"]["steps"])
    assert rep["collectives"] == {"skipped": "wall budget"}
    assert "skipped" in rep["c3_c4_engine_variants"]           # follows the skipped IPC core child
    assert rep["collectives_summary"]["ipc"] == {"skipped": "wall budget"}
