// msx_tree_sum.hip — k_tree launchers (SUM; the fp32 SUM tuning modes of msx_tune_tree), see msx_tree_impl.h.
#include "msx_tree_impl.h"

namespace msx {

template hipError_t tree_dispatch<O_SUM>(Kind, const dev::TreeArgs&, int, void*, size_t, hipStream_t);

// msx_tune_tree modes (fp32 SUM): 1/2/3 the generic kernel with
// loads up front / up front + non-temporal / interleaved + non-temporal,
// 4/5/6 the compile-time-source kernel with 1/2/4 vectors per lane, 7 = 5 with
// non-temporal loads, 8 the generic kernel as it is (the dispatch before the
// compile-time-source kernel); 9 = 4 with the tile order of the grid_cap
// argument (TreeArgs::xg: 0 XCD-contiguous, > 0 runs of that many tiles per
// XCD, -1 passed as 0x7fffffff: dispatch order, no grid cap in this mode),
// 10/11 = 4 with 512- / 1024-lane workgroups, 12/13 = 4/6 with non-temporal
// loads and 256-lane workgroups (p = 8 full trees only), 14 = 12 with mode 9's
// tile order, 15/16 = 12 with 64-lane workgroups in dispatch order (the
// default above tree_nt_min) / XCD-contiguous, 17 = the generic kernel in mode
// 15's geometry (its default above tree_nt_min); mode 0 (not routed here) is
// the default dispatch.
hipError_t tree_tune_f32_sum(int mode, const dev::TreeArgs& a, int ns, void* out, size_t n, hipStream_t s)
{
    switch (mode) {
    case 1: return run_tree<O_SUM, float, float, true, false>(a, ns, out, n, s);
    case 2: return run_tree<O_SUM, float, float, true, true>(a, ns, out, n, s);
    case 3: return run_tree<O_SUM, float, float, false, true>(a, ns, out, n, s);
    case 4: return run_tree_sel<O_SUM, float, float, 1, false>(a, ns, out, n, s);
    case 5: return run_tree_sel<O_SUM, float, float, 2, false>(a, ns, out, n, s);
    case 6: return run_tree_sel<O_SUM, float, float, 4, false>(a, ns, out, n, s);
    case 7: return run_tree_sel<O_SUM, float, float, 2, true>(a, ns, out, n, s);
    case 8: return run_tree<O_SUM, float, float>(a, ns, out, n, s);
    case 9: {
        TreeArgs b = a;
        b.xg = g_tree_tune.grid_cap == 0x7fffffff ? -1 : g_tree_tune.grid_cap;
        const int cap = g_tree_tune.grid_cap;
        g_tree_tune.grid_cap = 0;
        const hipError_t e = run_tree_sel<O_SUM, float, float, 1, false>(b, ns, out, n, s);
        g_tree_tune.grid_cap = cap;
        return e;
    }
    case 10:
    case 11:
        if (!a.chain && a.pairmask == 0 && a.nleaves == a.P && a.P == 8)
            return mode == 10 ? run_tree<O_SUM, float, float, false, false, 8, 1, false, 512>(a, ns, out, n, s)
                              : run_tree<O_SUM, float, float, false, false, 8, 1, false, 1024>(a, ns, out, n, s);
        return hipErrorInvalidValue;
    case 12:     // non-temporal loads, 256-lane workgroups (the DRAM-regime default before r03's one-wave form)
    case 14: {   // 12 with the tile order of the grid_cap argument (as mode 9)
        if (a.chain || a.pairmask != 0 || a.nleaves != a.P || a.P != 8) return hipErrorInvalidValue;
        TreeArgs b = a;
        if (mode == 14) b.xg = g_tree_tune.grid_cap == 0x7fffffff ? -1 : g_tree_tune.grid_cap;
        const int cap = g_tree_tune.grid_cap;
        g_tree_tune.grid_cap = 0;
        const hipError_t e = run_tree<O_SUM, float, float, false, true, 8, 1, false>(b, ns, out, n, s);
        g_tree_tune.grid_cap = cap;
        return e;
    }
    case 13: return run_tree_sel<O_SUM, float, float, 4, true>(a, ns, out, n, s);
    case 17: {   // the generic kernel, non-temporal loads, 64-lane workgroups in dispatch order
        TreeArgs b = a;
        b.xg = -1;
        return run_tree<O_SUM, float, float, false, true, 0, 1, false, 64>(b, ns, out, n, s);
    }
    case 15:     // 64-lane workgroups, non-temporal loads, dispatch order (k_combine_dram's geometry)
    case 16:     // 64-lane workgroups, non-temporal loads, XCD-contiguous
        if (!a.chain && a.pairmask == 0 && a.nleaves == a.P && a.P == 8) {
            TreeArgs b = a;
            b.xg = mode == 15 ? -1 : 0;
            return run_tree<O_SUM, float, float, false, true, 8, 1, false, 64>(b, ns, out, n, s);
        }
        return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
    }
}

}  // namespace msx
