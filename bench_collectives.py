#!/usr/bin/env python3
"""bench_collectives.py — the multi-rank configs of BASELINE.json, run by
bench.py at N > 1 as one child process per rank (so a failure here can never
take the headline local-reduce line down with it).

  c3  MPI_Allreduce      MPI_SUM  MPI_FLOAT     1 GiB per rank
  c4  MPI_Reduce_scatter MPI_MAX  MPI_DOUBLE    4 GiB sendbuf per rank, recvcount = total/p
  c5  MPI_Iallreduce     MPI_BAND MPI_UINT64_T  512 MiB, overlapped with a host compute loop
  + the §8f neighbours: MPI_Reduce (root 0, 1 GiB), MPI_Scan (64 MiB), one-sided
    MPI_Accumulate + MPI_Win_fence (256 MiB into the next rank's window)

Each rank is an MPI process of libmsmpi_mi355x.so (MSX_SIZE/MSX_RANK/MSX_DEVICE
set by the parent).  MSX_COLL_PARTS selects what runs, so bench.py can put the
headline configs first inside its wall budget: "core" = the all-peer write
probe + c3 + c4 + c5, "extras" = everything else, "c3c4" = c3 and c4 only (the
engine-variant run), "all" (default) = core, then extras.  Inputs are integer-valued patterns whose reductions are
exact in any order, so every result is checked in full on the GPU against a
closed form.  busBW = (S/t)·2(p−1)/p for allreduce, (S/t)·(p−1)/p for
reduce_scatter (S = bytes per rank).  Rank 0 writes one JSON object to the
path in argv[1].
"""
import ctypes
import json
import os
import re
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "microsoft-mpi_amd"))


def main(out_path, scale):
    import torch
    import msx

    L = msx.init(errors_return=True)
    C = msx.C
    r_, s_ = ctypes.c_int(), ctypes.c_int()
    L.MPI_Comm_rank(C.MPI_COMM_WORLD, ctypes.byref(r_))
    L.MPI_Comm_size(C.MPI_COMM_WORLD, ctypes.byref(s_))
    rank, p = r_.value, s_.value
    dev = torch.device("cuda", int(os.environ.get("MSX_DEVICE", "0")))
    torch.cuda.set_device(dev)
    # xGMI reference: 7 links x 153.6 GB/s bidirectional per MI355X = 76.8 GB/s
    # per direction per link; busBW (bytes each GPU moves per direction) is
    # compared with the 7-link per-direction aggregate
    XGMI = 7 * 76.8
    # Ranks sharing one GPU move every byte through that GPU's HBM: their busBW
    # is an HBM-plane figure, and no fraction of a link it never used is
    # emitted for them (the xGMI fields appear only with one rank per GPU).
    shared = L.msx_engine_gpu_shared() == 1
    res = {"ranks": p, "transport_requested": os.environ.get("MSX_TRANSPORT", "ipc"),
           "gpu_shared": shared, "plane": "hbm (ranks share one GPU)" if shared else "xgmi"}
    if not shared:
        res["xgmi_aggregate_GB_s_per_direction"] = XGMI

    def link_fracs(busbw, meas):
        """xGMI fractions of a busBW figure, for distinct GPUs only."""
        if shared:
            return {}
        return {"busbw_frac_xgmi": round(busbw / XGMI, 3),
                "busbw_frac_measured_links": round(busbw / meas, 3) if meas else None}
    logf = open(os.environ.get("MSX_BENCH_LOG", os.devnull), "a")

    def log(msg):
        logf.write(f"[{time.strftime('%H:%M:%S')}] rank {rank}: {msg}\n")
        logf.flush()

    log(f"init ok p={p} scale={scale}")
    part = os.environ.get("MSX_COLL_PARTS", "all")
    if part not in ("all", "core", "extras", "c3c4"):
        raise SystemExit(f"MSX_COLL_PARTS={part}")
    core, extras = part in ("all", "core", "c3c4"), part in ("all", "extras")
    res["parts"] = part
    # test hook (bench.py's wall-budget rehearsal): MSX_BENCH_TEST_HANG=
    # <transport>:<rank> makes that rank's child hang on the host, after
    # MPI_Init and before any collective, until bench.py's time limit kills it
    # (no GPU work in flight; its peers' waits run out first)
    if part != "extras" and os.environ.get("MSX_BENCH_TEST_HANG") == f"{res['transport_requested']}:{rank}":
        log("test hook: hanging")
        while True:
            time.sleep(1.0)

    def fail(config, rc):
        """Fail fast with a structured error: which config, and -- parsed from
        the library's timeout text (flag_timeout / ShmBarrier / Hub in
        msx_transport.cpp) -- which rank waited in which phase for which peer.
        Every rank writes <out>.rank<r>; the parent gathers them into its JSON
        line.  No MPI_Finalize: the peers may be gone."""
        text = msx.last_error()
        err = {"config": config, "rank": rank, "rc": rc, "text": text}
        m = re.search(r"(flag timeout|wait timeout|ipc error): op=(\S+) rank=(-?\d+) phase=(\S+) peer=(-?\d+)", text)
        if m:
            err.update({"kind": m.group(1), "op": m.group(2), "phase": m.group(4), "peer": int(m.group(5))})
        res["error"] = err
        log(f"FAILED {err}")
        for path in ([out_path] if rank == 0 else []) + [f"{out_path}.rank{rank}"]:
            with open(path, "w") as f:
                json.dump(res, f)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(3)

    def check(config, rc):
        if rc:
            fail(config, rc)
        return rc

    def barrier():
        check("barrier", L.MPI_Barrier(C.MPI_COMM_WORLD))

    xgmi_meas = None
    if core:
        # ---- c3: allreduce SUM fp32, 1 GiB per rank ------------------------------
        n = int((256 << 20) * scale)
        i = torch.arange(n, device=dev, dtype=torch.int64)
        send = (((i * 7 + rank * 13) % 17) - 8).to(torch.float32)
        recv = torch.empty_like(send)
        exp = torch.zeros(n, device=dev, dtype=torch.float32)
        for r in range(p):
            exp += (((i * 7 + r * 13) % 17) - 8).to(torch.float32)
        del i
        torch.cuda.synchronize()
        log("c3 data ready")
        # measured link roofline: every rank writes into all peers' windows at once
        # (the scatter step's pattern); busBW is also reported against it
        xgmi_meas = None
        if p > 1 and res["transport_requested"] == "ipc" and part != "c3c4":
            sec, used = ctypes.c_double(), ctypes.c_int64()
            rc = L.msx_peer_write_bandwidth(max(1 << 20, int((64 << 20) * scale)), 5, ctypes.byref(sec),
                                            ctypes.byref(used))
            if rc == 0 and sec.value > 0:
                xgmi_meas = (p - 1) * used.value / sec.value / 1e9
                res["peer_write_probe"] = {"bytes_per_peer": used.value, "seconds": round(sec.value, 6),
                                           "outbound_GB_s_per_gpu": round(xgmi_meas, 1),
                                           "plane": res["plane"]}
            else:
                res["peer_write_probe"] = {"error": f"rc={rc} {msx.last_error()}"}
            log(f"peer write probe {res['peer_write_probe']}")
        times = []
        stats = (ctypes.c_double * 7)()
        L.msx_engine_stats(stats, 7, 1)                 # reset the phase timers
        for it in range(4):
            if it == 1:
                L.msx_engine_stats(stats, 7, 1)         # phases of the timed calls only (not the warm-up's setup)
            barrier()
            t0 = time.perf_counter()
            rc = L.MPI_Allreduce(send.data_ptr(), recv.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM, C.MPI_COMM_WORLD)
            times.append(time.perf_counter() - t0)
            log(f"c3 iter {it} rc={rc} {times[-1]:.4f}s")
            if rc:
                fail("c3", rc)
                break
        if "c3_error" not in res:
            t = sorted(times[1:])[len(times[1:]) // 2]
            S = n * 4
            res["c3_allreduce_sum_f32"] = {
                "bytes_per_rank": S, "seconds": round(t, 5), "algbw_GB_s": round(S / t / 1e9, 2),
                "busbw_GB_s": round(S / t / 1e9 * 2 * (p - 1) / p, 2),
                **link_fracs(S / t / 1e9 * 2 * (p - 1) / p, xgmi_meas),
                "correct": bool(torch.equal(recv, exp))}
            L.msx_engine_stats(stats, 7, 1)
            calls = max(stats[6], 1.0)
            if stats[6] > 0:    # window plane only (the RCCL plane has no host phases)
                res["c3_allreduce_sum_f32"]["phase_ms_per_call"] = {
                    k: round(stats[i] / calls * 1e3, 3) for i, k in
                    enumerate(("stage_scatter", "collect_wait_barrier_a", "reduce_push", "barrier_b",
                               "final_collect"))}
                res["c3_allreduce_sum_f32"]["chunks_per_call"] = stats[5] / calls
        del send, recv, exp
        torch.cuda.empty_cache()

    # ---- c4: reduce_scatter MAX fp64, 4 GiB per rank sendbuf ----------------
    def c4_section():
        per = int((512 << 20) * scale) // p                  # recvcount per rank (c4: 2^29 / p)
        tot = per * p
        i = torch.arange(tot, device=dev, dtype=torch.int64)
        send = ((i * 2654435761 + rank * 40503) % 1000003).to(torch.float64)
        recv = torch.empty(per, device=dev, dtype=torch.float64)
        counts = (ctypes.c_int * p)(*([per] * p))
        lo, hi = rank * per, (rank + 1) * per
        ii = i[lo:hi]
        exp = torch.full((per,), -1.0, device=dev, dtype=torch.float64)
        for r in range(p):
            exp = torch.maximum(exp, ((ii * 2654435761 + r * 40503) % 1000003).to(torch.float64))
        del i, ii
        torch.cuda.synchronize()
        times = []
        for it in range(3):
            barrier()
            t0 = time.perf_counter()
            rc = L.MPI_Reduce_scatter(send.data_ptr(), recv.data_ptr(), counts, C.MPI_DOUBLE, C.MPI_MAX,
                                      C.MPI_COMM_WORLD)
            times.append(time.perf_counter() - t0)
            log(f"c4 iter {it} rc={rc} {times[-1]:.4f}s")
            if rc:
                fail("c4", rc)
                break
        if "c4_error" not in res:
            t = sorted(times[1:])[len(times[1:]) // 2]
            S = tot * 8
            res["c4_reduce_scatter_max_f64"] = {
                "bytes_per_rank": S, "seconds": round(t, 5), "busbw_GB_s": round(S / t / 1e9 * (p - 1) / p, 2),
                **link_fracs(S / t / 1e9 * (p - 1) / p, xgmi_meas),
                "correct": bool(torch.equal(recv, exp))}
        del send, recv, exp
        torch.cuda.empty_cache()

    if part == "c3c4":
        c4_section()
    elif core:
        c4_section()
        # ---- c5: iallreduce BAND u64, 512 MiB, overlapped with host compute ------
        n = int((64 << 20) * scale)
        i = torch.arange(n, device=dev, dtype=torch.int64)
        one = torch.ones((), dtype=torch.int64, device=dev)
        send = ~torch.bitwise_left_shift(one, (i + rank) % 64)          # all bits but one
        exp = torch.full((n,), -1, device=dev, dtype=torch.int64)
        for r in range(p):
            exp &= ~torch.bitwise_left_shift(one, (i + r) % 64)
        del i
        recv = torch.empty_like(send)
        import numpy as np
        host = np.random.default_rng(rank).random(1 << 20)

        def host_work(k):
            x = host
            for _ in range(k):
                x = x * 1.000001 + 0.5
            return x

        torch.cuda.synchronize()
        host_work(20)                                   # warm the host loop (page-in)
        rc = 0
        t_comm = 1e30
        for _ in range(2):
            barrier()
            t0 = time.perf_counter()
            rc = check("c5_blocking", L.MPI_Allreduce(send.data_ptr(), recv.data_ptr(), n, C.MPI_UINT64_T, C.MPI_BAND,
                                                      C.MPI_COMM_WORLD))
            t_comm = min(t_comm, time.perf_counter() - t0)
        # size the host loop to about the communication time, so the overlap is
        # measurable: efficiency = hidden time / min(t_comm, t_host), 1 = perfect
        t0 = time.perf_counter()
        host_work(20)
        per = (time.perf_counter() - t0) / 20
        K = max(1, int(round(t_comm / per)))
        t_host = 1e30
        for _ in range(2):
            t0 = time.perf_counter()
            host_work(K)
            t_host = min(t_host, time.perf_counter() - t0)
        # best of 3, like t_comm and t_host (one sample of a ~1 ms overlap on a
        # shared box varied 0.71-0.82 between runs)
        t_total, rc2, rc3 = 1e30, 0, 0
        for _ in range(3):
            barrier()
            req = ctypes.c_int()
            t0 = time.perf_counter()
            rc2 = rc2 or L.MPI_Iallreduce(send.data_ptr(), recv.data_ptr(), n, C.MPI_UINT64_T, C.MPI_BAND,
                                          C.MPI_COMM_WORLD, ctypes.byref(req))
            host_work(K)
            rc3 = rc3 or L.MPI_Wait(ctypes.byref(req), ctypes.c_void_p(1))
            t_total = min(t_total, time.perf_counter() - t0)
            if rc2 or rc3:
                break
        log(f"c5 done rc={rc},{rc2},{rc3} comm={t_comm:.4f} host={t_host:.4f} total={t_total:.4f}")
        if rc or rc2 or rc3:
            fail("c5", rc or rc2 or rc3)
        else:
            S = n * 8
            res["c5_iallreduce_band_u64"] = {
                "bytes_per_rank": S, "t_comm_s": round(t_comm, 5), "t_host_s": round(t_host, 5),
                "t_overlapped_s": round(t_total, 5),
                "busbw_GB_s": round(S / t_comm / 1e9 * 2 * (p - 1) / p, 2),
                **{k: v for k, v in link_fracs(S / t_comm / 1e9 * 2 * (p - 1) / p, xgmi_meas).items()
                   if k == "busbw_frac_measured_links"},
                "overlap_efficiency": round((t_comm + t_host - t_total) / min(t_comm, t_host), 3),
                "correct": bool(torch.equal(recv, exp))}
        del send, recv, exp
        torch.cuda.empty_cache()

    if extras:
        # allreduce latency / bandwidth curve (fp32 SUM, exact integer data)
        curve = {}
        for nbytes in (4 << 10, 256 << 10, 4 << 20, 64 << 20):
            m = nbytes // 4
            a, want = torch.ones(m, device=dev), torch.full((m,), float(p), device=dev)
            b = torch.empty_like(a)
            torch.cuda.synchronize()
            check(f"allreduce_curve_{nbytes}",
                  L.MPI_Allreduce(a.data_ptr(), b.data_ptr(), m, C.MPI_FLOAT, C.MPI_SUM, C.MPI_COMM_WORLD))
            # back-to-back calls after one barrier, averaged (the OSU latency
            # method: no barrier wake-up skew inside the timed calls)
            iters = 50 if nbytes <= (4 << 20) else 10
            ts = []
            for _ in range(3):
                barrier()
                t0 = time.perf_counter()
                for _ in range(iters):
                    check(f"allreduce_curve_{nbytes}",
                          L.MPI_Allreduce(a.data_ptr(), b.data_ptr(), m, C.MPI_FLOAT, C.MPI_SUM, C.MPI_COMM_WORLD))
                ts.append((time.perf_counter() - t0) / iters)
            t = sorted(ts)[1]
            curve[str(nbytes)] = {"us": round(t * 1e6, 1), "busbw_GB_s": round(nbytes / t / 1e9 * 2 * (p - 1) / p, 2),
                                  "correct": bool(torch.equal(b, want))}
        res["allreduce_curve_f32"] = curve
        # small rooted reduce latency (barrier-free binomial path), same method
        m = 1024
        a, out = torch.ones(m, device=dev), torch.zeros(m, device=dev)
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            barrier()
            t0 = time.perf_counter()
            for _ in range(50):
                check("reduce_4096B", L.MPI_Reduce(a.data_ptr(), out.data_ptr(), m, C.MPI_FLOAT, C.MPI_SUM, 0,
                                                   C.MPI_COMM_WORLD))
            ts.append((time.perf_counter() - t0) / 50)
        res["reduce_4096B_root0_us"] = {"us": round(sorted(ts)[1] * 1e6, 1),
                                         "correct": bool(torch.all(out == p).item()) if rank == 0 else None}

        # ---- c3 on host memory: the MPI path starts and ends in (pageable) host
        # buffers; 256 MiB per rank, PCIe-inclusive (pinned for the call and read /
        # written in place by the kernels)
        import numpy as np
        nh = int((64 << 20) * scale)
        ih = np.arange(nh, dtype=np.int64)
        hsend = (((ih * 7 + rank * 13) % 17) - 8).astype(np.float32)
        hexp = np.zeros(nh, np.float32)
        for r in range(p):
            hexp += (((ih * 7 + r * 13) % 17) - 8).astype(np.float32)
        del ih
        hrecv = np.empty_like(hsend)
        ts = []
        for it in range(4):
            barrier()
            t0 = time.perf_counter()
            rc = L.MPI_Allreduce(hsend.ctypes.data, hrecv.ctypes.data, nh, C.MPI_FLOAT, C.MPI_SUM, C.MPI_COMM_WORLD)
            ts.append(time.perf_counter() - t0)
            if rc:
                fail("c3_host", rc)
                break
        if "c3_host_error" not in res:
            t = sorted(ts[1:])[len(ts[1:]) // 2]
            res["c3_host_pageable_allreduce_sum_f32"] = {
                "bytes_per_rank": nh * 4, "seconds": round(t, 5), "algbw_GB_s": round(nh * 4 / t / 1e9, 2),
                "busbw_GB_s": round(nh * 4 / t / 1e9 * 2 * (p - 1) / p, 2),
                "correct": bool(np.array_equal(hrecv, hexp))}
        log(f"c3 host done {res.get('c3_host_pageable_allreduce_sum_f32', res.get('c3_host_error'))}")
        # the same on pinned (page-locked) host buffers, SURVEY 8(d)'s other host variant
        psend = torch.from_numpy(hsend).pin_memory()
        precv = torch.empty(nh, dtype=torch.float32).pin_memory()
        ts = []
        for it in range(4):
            barrier()
            t0 = time.perf_counter()
            rc = L.MPI_Allreduce(psend.data_ptr(), precv.data_ptr(), nh, C.MPI_FLOAT, C.MPI_SUM, C.MPI_COMM_WORLD)
            ts.append(time.perf_counter() - t0)
            if rc:
                fail("c3_host_pinned", rc)
                break
        if "c3_host_pinned_error" not in res:
            t = sorted(ts[1:])[len(ts[1:]) // 2]
            res["c3_host_pinned_allreduce_sum_f32"] = {
                "bytes_per_rank": nh * 4, "seconds": round(t, 5), "algbw_GB_s": round(nh * 4 / t / 1e9, 2),
                "busbw_GB_s": round(nh * 4 / t / 1e9 * 2 * (p - 1) / p, 2),
                "correct": bool(np.array_equal(precv.numpy(), hexp))}
        log(f"c3 pinned done {res.get('c3_host_pinned_allreduce_sum_f32', res.get('c3_host_pinned_error'))}")
        del hsend, hrecv, hexp, psend, precv

        # ---- c4 / c5 on host memory (the host variant of every GPU
        # config), at bounded sizes: a 512 MiB send buffer per rank for the
        # reduce_scatter MAX fp64, a 256 MiB uint64 vector for the Iallreduce BAND
        per_h = int((64 << 20) * scale) // p
        tot_h = per_h * p
        jh = np.arange(tot_h, dtype=np.int64)
        hs4 = ((jh * 2654435761 + rank * 40503) % 1000003).astype(np.float64)
        blk = jh[rank * per_h:(rank + 1) * per_h]
        he4 = np.full(per_h, -1.0)
        for r in range(p):
            he4 = np.maximum(he4, ((blk * 2654435761 + r * 40503) % 1000003).astype(np.float64))
        del jh, blk
        hr4 = np.empty(per_h, np.float64)
        hcounts = (ctypes.c_int * p)(*([per_h] * p))
        ts = []
        for it in range(3):
            barrier()
            t0 = time.perf_counter()
            rc = L.MPI_Reduce_scatter(hs4.ctypes.data, hr4.ctypes.data, hcounts, C.MPI_DOUBLE, C.MPI_MAX,
                                      C.MPI_COMM_WORLD)
            ts.append(time.perf_counter() - t0)
            if rc:
                fail("c4_host", rc)
                break
        if "c4_host_error" not in res:
            t = sorted(ts[1:])[len(ts[1:]) // 2]
            res["c4_host_pageable_reduce_scatter_max_f64"] = {
                "bytes_per_rank": tot_h * 8, "seconds": round(t, 5),
                "busbw_GB_s": round(tot_h * 8 / t / 1e9 * (p - 1) / p, 2),
                "correct": bool(np.array_equal(hr4, he4))}
        log(f"c4 host done {res.get('c4_host_pageable_reduce_scatter_max_f64', res.get('c4_host_error'))}")
        del hs4, hr4, he4
        n5 = int((32 << 20) * scale)
        k5 = np.arange(n5, dtype=np.uint64)
        bit = lambda r: np.left_shift(np.uint64(1), (k5 * np.uint64(7) + np.uint64(13 * r)) % np.uint64(64))
        hs5 = ~bit(rank)                                     # every rank clears one bit per element
        he5 = np.full(n5, np.uint64(0xFFFFFFFFFFFFFFFF))
        for r in range(p):
            he5 &= ~bit(r)
        del k5
        hr5 = np.empty_like(hs5)
        ts = []
        for it in range(3):
            barrier()
            req = ctypes.c_int()
            t0 = time.perf_counter()
            rc = L.MPI_Iallreduce(hs5.ctypes.data, hr5.ctypes.data, n5, C.MPI_UINT64_T, C.MPI_BAND, C.MPI_COMM_WORLD,
                                  ctypes.byref(req))
            rc = rc or L.MPI_Wait(ctypes.byref(req), ctypes.c_void_p(1))
            ts.append(time.perf_counter() - t0)
            if rc:
                fail("c5_host", rc)
                break
        if "c5_host_error" not in res:
            t = sorted(ts[1:])[len(ts[1:]) // 2]
            res["c5_host_pageable_iallreduce_band_u64"] = {
                "bytes_per_rank": n5 * 8, "seconds": round(t, 5),
                "busbw_GB_s": round(n5 * 8 / t / 1e9 * 2 * (p - 1) / p, 2),
                "correct": bool(np.array_equal(hr5, he5))}
        log(f"c5 host done {res.get('c5_host_pageable_iallreduce_band_u64', res.get('c5_host_error'))}")
        del hs5, hr5, he5

        # ---- §8f neighbours at the same measurement bar -------------------------
        def timed(fn, reps=3):
            ts = []
            for _ in range(reps + 1):
                barrier()
                t0 = time.perf_counter()
                rc = fn()
                ts.append(time.perf_counter() - t0)
                if rc:
                    return None, rc
            return sorted(ts[1:])[len(ts[1:]) // 2], 0

        # MPI_Reduce SUM fp32 at root 0 (Rabenseifner reduce-scatter + gather),
        # 1 GiB per rank like c3
        n = int((256 << 20) * scale)
        i = torch.arange(n, device=dev, dtype=torch.int64)
        send = (((i * 5 + rank * 3) % 13) - 6).to(torch.float32)
        exp = torch.zeros(n, device=dev, dtype=torch.float32)
        for r in range(p):
            exp += (((i * 5 + r * 3) % 13) - 6).to(torch.float32)
        del i
        recv = torch.zeros_like(send)
        torch.cuda.synchronize()
        t, rc = timed(lambda: L.MPI_Reduce(send.data_ptr(), recv.data_ptr(), n, C.MPI_FLOAT, C.MPI_SUM, 0,
                                           C.MPI_COMM_WORLD))
        if rc:
            fail("reduce", rc)
        else:
            S = n * 4
            res["reduce_sum_f32_root0"] = {"bytes_per_rank": S, "seconds": round(t, 5),
                                           "busbw_GB_s": round(S / t / 1e9 * (p - 1) / p, 2),
                                           "correct": bool(torch.equal(recv, exp)) if rank == 0 else None}
        # MPI_Scan SUM fp32, 64 MiB per rank (recursive-doubling task order)
        m = int((16 << 20) * max(scale, 1.0 / 16))
        send2 = send[:m].clone()
        pre = torch.zeros(m, device=dev, dtype=torch.float32)
        i = torch.arange(m, device=dev, dtype=torch.int64)
        for r in range(rank + 1):
            pre += (((i * 5 + r * 3) % 13) - 6).to(torch.float32)
        del i
        out = torch.zeros_like(send2)
        torch.cuda.synchronize()
        t, rc = timed(lambda: L.MPI_Scan(send2.data_ptr(), out.data_ptr(), m, C.MPI_FLOAT, C.MPI_SUM,
                                         C.MPI_COMM_WORLD))
        if rc:
            fail("scan", rc)
        else:
            res["scan_sum_f32"] = {"bytes_per_rank": m * 4, "seconds": round(t, 5),
                                   "GB_s_per_rank": round(m * 4 / t / 1e9, 2), "correct": bool(torch.equal(out, pre))}
        del send, recv, exp, send2, pre, out
        torch.cuda.empty_cache()

        # one-sided MPI_Accumulate SUM fp32: every rank adds 256 MiB into the next
        # rank's device window; a fence closes the epoch (target-side application)
        n = int((64 << 20) * max(scale, 1.0 / 16))
        base = torch.full((n,), 1.0, device=dev)
        contrib = torch.full((n,), float(rank + 1), device=dev)
        torch.cuda.synchronize()
        win = ctypes.c_int()
        rc = L.MPI_Win_create(base.data_ptr(), n * 4, 4, C.MPI_INFO_NULL, C.MPI_COMM_WORLD, ctypes.byref(win))
        if not rc:
            rc = L.MPI_Win_fence(0, win)
        reps = 3
        if not rc:
            tgt = (rank + 1) % p
            ts = []
            for _ in range(reps + 1):
                barrier()
                t0 = time.perf_counter()
                rc = L.MPI_Accumulate(contrib.data_ptr(), n, C.MPI_FLOAT, tgt, 0, n, C.MPI_FLOAT, C.MPI_SUM, win) or \
                    L.MPI_Win_fence(0, win)
                ts.append(time.perf_counter() - t0)
                if rc:
                    break
        if rc:
            fail("rma", rc)
        else:
            t = sorted(ts[1:])[len(ts[1:]) // 2]
            src_rank = (rank - 1) % p
            res["rma_accumulate_sum_f32_fence"] = {
                "bytes_per_rank": n * 4, "seconds": round(t, 5), "GB_s_per_rank": round(n * 4 / t / 1e9, 2),
                "correct": bool(torch.all(base == 1.0 + (reps + 1) * (src_rank + 1)).item())}
            done = 1.0 + (reps + 1) * (src_rank + 1)

            # the same accumulate in a passive-target epoch (lock / unlock: the
            # target's service thread applies it) and in a post-start-complete-wait
            # epoch with the ring's neighbours
            def passive():
                return (L.MPI_Win_lock(C.MPI_LOCK_SHARED, tgt, 0, win) or
                        L.MPI_Accumulate(contrib.data_ptr(), n, C.MPI_FLOAT, tgt, 0, n, C.MPI_FLOAT, C.MPI_SUM, win) or
                        L.MPI_Win_unlock(tgt, win))
            wg = ctypes.c_int()
            L.MPI_Comm_group(C.MPI_COMM_WORLD, ctypes.byref(wg))
            gprev, gnext = ctypes.c_int(), ctypes.c_int()
            L.MPI_Group_incl(wg.value, 1, (ctypes.c_int * 1)(src_rank), ctypes.byref(gprev))
            L.MPI_Group_incl(wg.value, 1, (ctypes.c_int * 1)(tgt), ctypes.byref(gnext))

            def pscw():
                return (L.MPI_Win_post(gprev.value, 0, win) or L.MPI_Win_start(gnext.value, 0, win) or
                        L.MPI_Accumulate(contrib.data_ptr(), n, C.MPI_FLOAT, tgt, 0, n, C.MPI_FLOAT, C.MPI_SUM, win) or
                        L.MPI_Win_complete(win) or L.MPI_Win_wait(win))
            for key, fn in (("rma_accumulate_sum_f32_lock", passive), ("rma_accumulate_sum_f32_pscw", pscw)):
                t, rc = timed(fn)
                if rc:
                    fail(key, rc)
                    break
                barrier()
                done += (3 + 1) * (src_rank + 1)
                res[key] = {"bytes_per_rank": n * 4, "seconds": round(t, 5), "GB_s_per_rank": round(n * 4 / t / 1e9, 2),
                            "correct": bool(torch.all(base == done).item())}
            for g in (gprev, gnext, wg):
                L.MPI_Group_free(ctypes.byref(g))
            L.MPI_Win_free(ctypes.byref(win))
    barrier()
    L.msx_engine_transport.restype = ctypes.c_char_p
    res["transport_used"] = L.msx_engine_transport().decode()
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(res, f)
    L.MPI_Finalize()


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 1.0)
