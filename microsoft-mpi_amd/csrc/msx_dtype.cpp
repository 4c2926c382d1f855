// msx_dtype.cpp — derived datatypes (see msx_dtype.h).
//
// Type attributes follow the reference's constructors exactly:
//   MPID_Type_vector        datatype.cpp:2495-2622 (also contiguous/hvector)
//   MPID_Type_indexed       datatype.cpp:1870-2060 (also hindexed, *_block)
//   MPID_Type_struct        datatype.cpp:2214-2473 (sticky LB/UB, alignment pad)
//   MPID_Type_create_resized datatype.cpp:1417-1493
//   MPID_Type_zerolen       datatype.cpp:2639-2683
//   pair types              datatype.cpp:1282-1413 (size != extent)
//   builtin attributes      datatype.cpp:222-306
//   MPID_Type_convert_subarray datatype.cpp:3274-3399
//   LB/UB helpers           include/datatype.h:522-611
// The type map itself is kept flattened (ordered byte runs of one instance);
// the GPU kernels in msx_pack.hip move the bytes.
#include "msx_dtype.h"

#include <string.h>

#include <algorithm>
#include <map>
#include <memory>

#include "msx_comm.h"
#include "msx_runtime.h"

namespace msx {

hipError_t launch_dt_copy(const DevLayout& L, int64_t count, void* typed, void* packed, bool unpack,
                          hipStream_t s);
hipError_t launch_dt_acc(int opidx, Kind k, const DevLayout& L, int64_t count, const void* packed,
                         void* typed, hipStream_t s);

namespace {

constexpr int64_t kMaxRuns = (int64_t)1 << 25;     // explicit runs kept per type

// Two-level compact forms (Dtype::rn2); MSX_TEST_DT_COMPACT2=0 expands them into
// explicit run lists as before (A/B and fallback).
bool compact2_enabled()
{
    static const bool on = [] {
        const char* e = getenv("MSX_TEST_DT_COMPACT2");
        return !e || atoi(e) != 0;
    }();
    return on;
}
constexpr int kPairSlots = 5;                       // direct slots 0..4: MPI_FLOAT_INT .. MPI_LONG_DOUBLE_INT
constexpr unsigned kDirectTypeBits = 0x8c000000u;   // HANDLE_TYPE_DIRECT | MPID_DATATYPE

std::recursive_mutex g_mu;
std::vector<Dtype*> g_slots;                        // derived types by direct index
std::map<MPI_Datatype, std::unique_ptr<Dtype>> g_predef;

int64_t lowbit_align(int64_t v)
{
    uint64_t u = (uint64_t)(v < 0 ? -v : v);
    if (u == 0) return 16;
    int64_t a = (int64_t)(u & (~u + 1));
    return a > 16 ? 16 : a;
}

// ---- predefined types --------------------------------------------------------
int builtin_alignsize(MPI_Datatype d, int64_t size)
{
    switch (d) {
    case MPI_2INTEGER: case MPI_2INT: return 4;
    case MPI_2REAL: case MPI_COMPLEX: case MPI_2COMPLEX: case MPI_COMPLEX8: case MPI_C_COMPLEX:
    case MPI_C_FLOAT_COMPLEX: return 4;
    case MPI_DOUBLE_COMPLEX: case MPI_2DOUBLE_PRECISION: case MPI_2DOUBLE_COMPLEX: case MPI_COMPLEX16:
    case MPI_C_DOUBLE_COMPLEX: case MPI_C_LONG_DOUBLE_COMPLEX: return 8;
    default: return (int)size;
    }
}

// SetTypeCharacteristics<T1,T2> (datatype.cpp:1282-1293) with the LLP64 sizes:
// long = 4, long double = double.
bool pair_layout(MPI_Datatype d, int64_t* s1, int64_t* s2, int64_t* off2, int64_t* ext, int64_t* al)
{
    switch (d) {
    case MPI_FLOAT_INT: *s1 = 4; *s2 = 4; *off2 = 4; *ext = 8; *al = 4; return true;
    case MPI_DOUBLE_INT: *s1 = 8; *s2 = 4; *off2 = 8; *ext = 16; *al = 8; return true;
    case MPI_LONG_INT: *s1 = 4; *s2 = 4; *off2 = 4; *ext = 8; *al = 4; return true;
    case MPI_SHORT_INT: *s1 = 2; *s2 = 4; *off2 = 4; *ext = 8; *al = 4; return true;
    case MPI_LONG_DOUBLE_INT: *s1 = 8; *s2 = 4; *off2 = 8; *ext = 16; *al = 8; return true;
    default: return false;
    }
}

void push_run(std::vector<DtRun>& out, int64_t disp, int64_t len)
{
    if (len <= 0) return;
    if (!out.empty() && out.back().disp + out.back().len == disp) {
        out.back().len += len;
        return;
    }
    out.push_back({disp, len});
}

Dtype* make_predef(MPI_Datatype d)
{
    int64_t s1, s2, off2, ext, al;
    auto t = std::make_unique<Dtype>();
    t->handle = d;
    t->permanent = true;
    t->committed = true;
    if (pair_layout(d, &s1, &s2, &off2, &ext, &al)) {
        t->size = s1 + s2;
        t->extent = ext;
        t->lb = 0;
        t->ub = ext;
        t->true_lb = 0;
        t->true_ub = off2 + s2;
        t->alignsize = al;
        t->eltype = MPI_DATATYPE_NULL;
        t->el_size = (s1 == s2) ? s1 : -1;
        t->n_elements = 2;
        t->is_contig = (t->size == t->extent);
        push_run(t->runs, 0, s1);
        push_run(t->runs, off2, s2);
    } else {
        if (handle_type(d) != HT_BUILTIN) return nullptr;
        const int sz = type_size(d);
        if (sz < 0) return nullptr;
        t->size = sz;
        t->extent = sz;
        t->ub = sz;
        t->true_ub = sz;
        t->alignsize = builtin_alignsize(d, sz);
        t->eltype = d;
        t->el_size = sz;
        t->n_elements = 1;
        t->is_contig = true;
        push_run(t->runs, 0, sz);
    }
    Dtype* p = t.get();
    g_predef[d] = std::move(t);
    return p;
}

Dtype* lookup_locked(MPI_Datatype h)
{
    if (h == MPI_DATATYPE_NULL) return nullptr;
    const unsigned u = (unsigned)h;
    if ((u & 0xfc000000u) == kDirectTypeBits) {
        const size_t idx = u & 0x03ffffffu;
        if (idx >= (size_t)kPairSlots) return idx < g_slots.size() ? g_slots[idx] : nullptr;
    }
    auto it = g_predef.find(h);
    if (it != g_predef.end()) return it->second.get();
    return make_predef(h);
}

MPI_Datatype register_type(std::unique_ptr<Dtype> t)
{
    if (g_slots.size() < (size_t)kPairSlots) g_slots.resize(kPairSlots, nullptr);
    size_t idx = kPairSlots;
    while (idx < g_slots.size() && g_slots[idx]) ++idx;
    if (idx == g_slots.size()) g_slots.push_back(nullptr);
    t->handle = (MPI_Datatype)(kDirectTypeBits | (unsigned)idx);
    // the contents hold a reference on every derived type they name
    for (MPI_Datatype h : t->types)
        if (Dtype* o = (dtype_is_derived(h) ? lookup_locked(h) : nullptr)) o->refs++;
    g_slots[idx] = t.release();
    return g_slots[idx]->handle;
}

void destroy(Dtype* t)
{
    if (t->dev_mem) (void)hipFree(t->dev_mem);
    delete t;
}

// The single run of a one-run type (either form).
bool single_run(const Dtype* t, DtRun* r)
{
    if (t->rn == 1 && t->rn2 == 1) { *r = {t->rfirst, t->rlen}; return true; }
    if (t->rn == 0 && t->runs.size() == 1) { *r = t->runs[0]; return true; }
    return false;
}

void copy_layout(Dtype* t, const Dtype* o)
{
    t->runs = o->runs;
    t->rn = o->rn;
    t->rfirst = o->rfirst;
    t->rlen = o->rlen;
    t->rstride = o->rstride;
    t->rn2 = o->rn2;
    t->rstride2 = o->rstride2;
}

// Append `nrep` copies of old's runs, copy r at disp0 + r*ext.  A compact old
// type is expanded into a local list: committed types are never modified (a
// pack may be reading them on another thread).
int append_copies(std::vector<DtRun>& out, const Dtype* old, int64_t disp0, int64_t nrep, int64_t ext)
{
    std::vector<DtRun> expanded;
    const std::vector<DtRun>* runs = &old->runs;
    if (old->rn) {
        if (old->rn > kMaxRuns / old->rn2) {
            set_error("datatype type map exceeds %lld contiguous pieces", (long long)kMaxRuns);
            return MPI_ERR_NO_MEM;
        }
        expanded.reserve((size_t)(old->rn * old->rn2));
        dtype_for_each_run(old, [&](int64_t d, int64_t l) { push_run(expanded, d, l); });
        runs = &expanded;
    }
    if (nrep <= 0 || runs->empty()) return MPI_SUCCESS;
    // one contiguous run spanning exactly the extent: the copies merge into one
    if (runs->size() == 1 && (*runs)[0].len == ext && ext > 0) {
        push_run(out, disp0 + (*runs)[0].disp, nrep * ext);
        return MPI_SUCCESS;
    }
    if ((int64_t)out.size() + nrep * (int64_t)runs->size() > kMaxRuns) {
        set_error("datatype type map exceeds %lld contiguous pieces", (long long)kMaxRuns);
        return MPI_ERR_NO_MEM;
    }
    for (int64_t r = 0; r < nrep; ++r)
        for (const DtRun& x : *runs) push_run(out, disp0 + r * ext + x.disp, x.len);
    return MPI_SUCCESS;
}

// MPID_DATATYPE_BLOCK_LB_UB (datatype.h:591-611)
void block_lb_ub(int64_t cnt, int64_t disp, int64_t olb, int64_t oub, int64_t oext, int64_t* lb, int64_t* ub)
{
    if (cnt == 0) { *lb = olb + disp; *ub = oub + disp; }
    else if (oub >= olb) { *lb = olb + disp; *ub = oub + disp + oext * (cnt - 1); }
    else { *lb = olb + disp + oext * (cnt - 1); *ub = oub + disp; }
}

// MPID_DATATYPE_VECTOR_LB_UB (datatype.h:549-580)
void vector_lb_ub(int64_t cnt, int64_t stride, int64_t blk, int64_t olb, int64_t oub, int64_t oext, int64_t* lb,
                  int64_t* ub)
{
    if (cnt == 0 || blk == 0) { *lb = olb; *ub = oub; }
    else if (stride >= 0 && oext >= 0) { *lb = olb; *ub = oub + oext * (blk - 1) + stride * (cnt - 1); }
    else if (stride < 0 && oext >= 0) { *lb = olb + stride * (cnt - 1); *ub = oub + oext * (blk - 1); }
    else if (stride >= 0 && oext < 0) { *lb = olb + oext * (blk - 1); *ub = oub + stride * (cnt - 1); }
    else { *lb = olb + oext * (blk - 1) + stride * (cnt - 1); *ub = oub; }
}

// MPID_Type_zerolen
std::unique_ptr<Dtype> zerolen()
{
    auto t = std::make_unique<Dtype>();
    t->is_contig = true;
    t->eltype = MPI_DATATYPE_NULL;
    return t;
}

bool is_builtin_h(MPI_Datatype h) { return handle_type(h) == HT_BUILTIN; }

// old-type attributes as the constructors read them (builtins: basic size)
struct Old {
    int64_t lb, ub, extent, true_lb, true_ub, size, el_size, n_el, alignsize;
    MPI_Datatype eltype;
    bool contig, sticky_lb, sticky_ub;
};
Old old_attrs(const Dtype* o, bool builtin)
{
    Old r;
    r.lb = builtin ? 0 : o->lb;
    r.ub = builtin ? o->size : o->ub;
    r.extent = builtin ? o->size : o->extent;
    r.true_lb = builtin ? 0 : o->true_lb;
    r.true_ub = builtin ? o->size : o->true_ub;
    r.size = o->size;
    r.el_size = builtin ? o->size : o->el_size;
    r.n_el = builtin ? 1 : o->n_elements;
    r.eltype = builtin ? o->handle : o->eltype;
    r.alignsize = builtin ? o->size : o->alignsize;
    r.contig = builtin ? true : o->is_contig;
    r.sticky_lb = builtin ? false : o->sticky_lb;
    r.sticky_ub = builtin ? false : o->sticky_ub;
    return r;
}

void set_contents(Dtype* t, int combiner, std::vector<int> ints, std::vector<MPI_Aint> aints,
                  std::vector<MPI_Datatype> types)
{
    t->combiner = combiner;
    t->ints = std::move(ints);
    t->aints = std::move(aints);
    t->types = std::move(types);
}

}  // namespace

// ---------------------------------------------------------------------------
Dtype* dtype_lookup(MPI_Datatype h)
{
    std::lock_guard<std::recursive_mutex> g(g_mu);
    return lookup_locked(h);
}

bool dtype_is_derived(MPI_Datatype h)
{
    const unsigned u = (unsigned)h;
    return (u & 0xfc000000u) == kDirectTypeBits && (u & 0x03ffffffu) >= (unsigned)kPairSlots;
}

int64_t dtype_size(MPI_Datatype h)
{
    Dtype* t = dtype_lookup(h);
    return t ? t->size : -1;
}

int64_t dtype_nruns(const Dtype* t) { return t->rn ? t->rn * t->rn2 : (int64_t)t->runs.size(); }

void dtype_add_ref(MPI_Datatype h)
{
    std::lock_guard<std::recursive_mutex> g(g_mu);
    if (!dtype_is_derived(h)) return;
    if (Dtype* t = lookup_locked(h)) t->refs++;
}

// MPID_Type_vector (strideinbytes selects hvector); contiguous = vector(count,
// 1, extent) in its LB/UB (MPID_DATATYPE_CONTIG_LB_UB gives the same values).
int dtype_vector(int count, int blocklen, int64_t stride, bool stride_bytes, MPI_Datatype oldh,
                 MPI_Datatype* out, int combiner)
{
    std::lock_guard<std::recursive_mutex> g(g_mu);
    Dtype* o = lookup_locked(oldh);
    if (!o) { set_error("invalid oldtype 0x%x", oldh); return MPI_ERR_TYPE; }
    std::unique_ptr<Dtype> t;
    if (count == 0) {
        t = zerolen();
    } else {
        const bool bi = is_builtin_h(oldh);
        const Old a = old_attrs(o, bi);
        t = std::make_unique<Dtype>();
        const int64_t eff = stride_bytes ? stride : stride * a.extent;
        t->size = (int64_t)count * blocklen * a.size;
        t->sticky_lb = a.sticky_lb;
        t->sticky_ub = a.sticky_ub;
        t->alignsize = a.alignsize;
        t->n_elements = (int64_t)count * blocklen * a.n_el;
        t->el_size = a.el_size;
        t->eltype = a.eltype;
        vector_lb_ub(count, eff, blocklen, a.lb, a.ub, a.extent, &t->lb, &t->ub);
        t->true_lb = t->lb + (a.true_lb - a.lb);
        t->true_ub = t->ub + (a.true_ub - a.ub);
        t->extent = t->ub - t->lb;
        t->is_contig = (t->size == t->extent && eff == (int64_t)blocklen * a.size && a.contig);
        // a one-run old type whose `blocklen` copies merge into one run gives a
        // regular run list: keep it compact (merged into one run if contiguous)
        DtRun r1;
        const bool one = blocklen > 0 && single_run(o, &r1) && (blocklen == 1 || r1.len == a.extent);
        const int64_t blen = one ? (blocklen == 1 ? r1.len : (int64_t)blocklen * a.extent) : 0;
        if (one && blen > 0 && eff == blen) {
            push_run(t->runs, r1.disp, (int64_t)count * blen);
        } else if (one && blen > 0 && count > 1) {
            t->rn = count;
            t->rfirst = r1.disp;
            t->rlen = blen;
            t->rstride = eff;
        } else if (blocklen == 1 && count > 1 && o->rn > 1 && o->rn2 == 1 && compact2_enabled()) {
            // one copy per block of a one-level compact type: two levels
            t->rn = o->rn;
            t->rfirst = o->rfirst;
            t->rlen = o->rlen;
            t->rstride = o->rstride;
            t->rn2 = count;
            t->rstride2 = eff;
        } else {
            for (int j = 0; j < count; ++j) {
                int rc = append_copies(t->runs, o, (int64_t)j * eff, blocklen, a.extent);
                if (rc != MPI_SUCCESS) return rc;
            }
        }
    }
    if (combiner == 3)          // MPI_COMBINER_CONTIGUOUS
        set_contents(t.get(), combiner, {count}, {}, {oldh});
    else if (combiner == 4)     // MPI_COMBINER_VECTOR
        set_contents(t.get(), combiner, {count, blocklen, (int)stride}, {}, {oldh});
    else                        // MPI_COMBINER_HVECTOR[_INTEGER]
        set_contents(t.get(), combiner, {count, blocklen}, {stride}, {oldh});
    *out = register_type(std::move(t));
    return MPI_SUCCESS;
}

int dtype_contiguous(int count, MPI_Datatype oldh, MPI_Datatype* out)
{
    std::lock_guard<std::recursive_mutex> g(g_mu);
    Dtype* o = lookup_locked(oldh);
    if (!o) { set_error("invalid oldtype 0x%x", oldh); return MPI_ERR_TYPE; }
    const int64_t ext = is_builtin_h(oldh) ? o->size : o->extent;
    return dtype_vector(count, 1, ext, true, oldh, out, 3);
}

// MPID_Type_indexed (datatype.cpp:1870-2060); `disps` are ints in old extents
// (indexed) or MPI_Aint bytes (hindexed).
int dtype_indexed(int count, const int* blens, const void* disps, bool disp_bytes, MPI_Datatype oldh,
                  MPI_Datatype* out, int combiner)
{
    std::lock_guard<std::recursive_mutex> g(g_mu);
    Dtype* o = lookup_locked(oldh);
    if (!o) { set_error("invalid oldtype 0x%x", oldh); return MPI_ERR_TYPE; }
    const bool bi = is_builtin_h(oldh);
    const Old a = old_attrs(o, bi);
    auto eff_disp = [&](int i) -> int64_t {
        return disp_bytes ? static_cast<const MPI_Aint*>(disps)[i]
                          : (int64_t) static_cast<const int*>(disps)[i] * a.extent;
    };
    int first_nz = 0;
    while (first_nz < count && blens[first_nz] == 0) ++first_nz;
    std::unique_ptr<Dtype> t;
    if (first_nz == count) {
        t = zerolen();
    } else {
        t = std::make_unique<Dtype>();
        t->sticky_lb = a.sticky_lb;
        t->sticky_ub = a.sticky_ub;
        t->alignsize = a.alignsize;
        t->el_size = a.el_size;
        t->eltype = a.eltype;
        int64_t old_ct = blens[first_nz], min_lb, max_ub;
        block_lb_ub(blens[first_nz], eff_disp(first_nz), a.lb, a.ub, a.extent, &min_lb, &max_ub);
        for (int i = first_nz + 1; i < count; ++i) {
            if (blens[i] <= 0) continue;
            old_ct += blens[i];
            int64_t l, u;
            block_lb_ub(blens[i], eff_disp(i), a.lb, a.ub, a.extent, &l, &u);
            min_lb = std::min(min_lb, l);
            max_ub = std::max(max_ub, u);
        }
        t->size = old_ct * a.size;
        t->lb = min_lb;
        t->ub = max_ub;
        t->true_lb = min_lb + (a.true_lb - a.lb);
        t->true_ub = max_ub + (a.true_ub - a.ub);
        t->extent = max_ub - min_lb;
        t->n_elements = old_ct * a.n_el;
        for (int i = 0; i < count; ++i) {
            int rc = append_copies(t->runs, o, eff_disp(i), blens[i], a.extent);
            if (rc != MPI_SUCCESS) return rc;
        }
        t->is_contig = a.contig && t->runs.size() == 1 && t->size == t->extent;
    }
    std::vector<int> ints{count};
    ints.insert(ints.end(), blens, blens + count);
    if (disp_bytes) {
        const MPI_Aint* d = static_cast<const MPI_Aint*>(disps);
        set_contents(t.get(), combiner, ints, std::vector<MPI_Aint>(d, d + count), {oldh});
    } else {
        const int* d = static_cast<const int*>(disps);
        ints.insert(ints.end(), d, d + count);
        set_contents(t.get(), combiner, ints, {}, {oldh});
    }
    *out = register_type(std::move(t));
    return MPI_SUCCESS;
}

int dtype_indexed_block(int count, int blen, const void* disps, bool disp_bytes, MPI_Datatype oldh,
                        MPI_Datatype* out, int combiner)
{
    std::vector<int> blens((size_t)std::max(count, 0), blen);
    int rc = dtype_indexed(count, blens.data(), disps, disp_bytes, oldh, out, combiner);
    if (rc != MPI_SUCCESS) return rc;
    std::lock_guard<std::recursive_mutex> g(g_mu);
    Dtype* t = lookup_locked(*out);
    std::vector<int> ints{count, blen};
    if (disp_bytes) {
        set_contents(t, combiner, ints, t->aints, {oldh});
    } else {
        const int* d = static_cast<const int*>(disps);
        ints.insert(ints.end(), d, d + count);
        set_contents(t, combiner, ints, {}, {oldh});
    }
    return MPI_SUCCESS;
}

// MPID_Type_struct (datatype.cpp:2214-2473) with MPID_Type_struct_alignsize.
int dtype_struct(int count, const int* blens, const MPI_Aint* disps, const MPI_Datatype* types,
                 MPI_Datatype* out, int combiner)
{
    std::lock_guard<std::recursive_mutex> g(g_mu);
    std::vector<Dtype*> olds((size_t)std::max(count, 0));
    for (int i = 0; i < count; ++i) {
        olds[i] = lookup_locked(types[i]);
        if (!olds[i]) { set_error("invalid datatype 0x%x in struct", types[i]); return MPI_ERR_TYPE; }
    }
    int i = 0;
    while (i < count && blens[i] == 0) ++i;
    std::unique_ptr<Dtype> t;
    if (count == 0 || i == count) {
        t = zerolen();
    } else {
        t = std::make_unique<Dtype>();
        bool found_slb = false, found_sub = false, found_tlb = false, found_tub = false, found_el = false;
        int64_t el_sz = 0, size = 0, tlb = 0, tub = 0, slb = 0, sub = 0, n_el = 0;
        // One real entry of one copy of a compact type among LB/UB markers
        // (MPI_Type_create_subarray / darray's closing struct): the layout
        // stays compact, shifted by the entry's displacement.
        int n_real = 0, sole = -1;
        for (int k = 0; k < count; ++k)
            if (blens[k] != 0 && types[k] != MPI_LB && types[k] != MPI_UB) { ++n_real; sole = k; }
        const bool keep_compact = n_real == 1 && blens[sole] == 1 && !is_builtin_h(types[sole]) && olds[sole]->rn > 0;
        MPI_Datatype el_type = MPI_DATATYPE_NULL;
        for (i = 0; i < count; ++i) {
            if (blens[i] == 0) continue;
            const bool bi = is_builtin_h(types[i]);
            const Dtype* o = olds[i];
            const bool marker = (types[i] == MPI_LB || types[i] == MPI_UB);
            int64_t l, u, tl, tu, esz;
            MPI_Datatype et;
            if (bi) {
                esz = o->size;
                et = types[i];
                block_lb_ub(blens[i], disps[i], 0, esz, esz, &l, &u);
                tl = l;
                tu = u;
                size += esz * blens[i];
                n_el += blens[i];
            } else {
                esz = o->el_size;
                et = o->eltype;
                block_lb_ub(blens[i], disps[i], o->lb, o->ub, o->extent, &l, &u);
                tl = l + (o->true_lb - o->lb);
                tu = u + (o->true_ub - o->ub);
                size += o->size * blens[i];
                n_el += o->n_elements * blens[i];
            }
            if (!marker) {
                if (!found_el) { el_sz = esz; el_type = et; found_el = true; }
                else if (el_sz != esz) { el_sz = -1; el_type = MPI_DATATYPE_NULL; }
                else if (el_type != et) { el_type = MPI_DATATYPE_NULL; }
            }
            if (types[i] == MPI_LB || (!bi && o->sticky_lb)) {
                if (!found_slb) { found_slb = true; slb = l; }
                else if (slb > l) slb = l;
            }
            if (types[i] == MPI_UB || (!bi && o->sticky_ub)) {
                if (!found_sub) { found_sub = true; sub = u; }
                else if (sub < u) sub = u;
            }
            if (!marker) {
                if (!found_tlb) { found_tlb = true; tlb = tl; }
                else if (tlb > tl) tlb = tl;
                if (!found_tub) { found_tub = true; tub = tu; }
                else if (tub < tu) tub = tu;
            }
            if (!marker && keep_compact) {
                copy_layout(t.get(), o);
                t->rfirst += disps[i];
            } else if (!marker) {
                const int64_t oext = bi ? o->size : o->extent;
                int rc = append_copies(t->runs, o, disps[i], blens[i], oext);
                if (rc != MPI_SUCCESS) return rc;
            }
        }
        t->n_elements = n_el;
        t->el_size = el_sz;
        t->eltype = el_type;
        t->sticky_lb = found_slb;
        t->true_lb = tlb;
        t->lb = found_slb ? slb : tlb;
        t->sticky_ub = found_sub;
        t->true_ub = tub;
        t->ub = found_sub ? sub : tub;
        // MPID_Type_struct_alignsize (datatype.cpp:2149-2195)
        int64_t maxal = 0;
        for (int k = 0; k < count; ++k) {
            if (types[k] == MPI_LB || types[k] == MPI_UB) continue;
            int64_t al = olds[k]->alignsize;
            if (al == 0) continue;
            const int64_t un = disps[k] % al;
            if (un != 0) {
                uint64_t x = (uint64_t)un;
                al = (int64_t)(x & (~x + 1));      // lowest set bit (_BitScanForward)
            }
            maxal = std::max(maxal, al);
        }
        t->alignsize = maxal;
        t->extent = t->ub - t->lb;
        if (!found_slb && !found_sub) {
            const int64_t eps = t->alignsize > 0 ? t->extent % t->alignsize : 0;
            if (eps) {
                t->ub += t->alignsize - eps;
                t->extent = t->ub - t->lb;
            }
        }
        t->size = size;
        t->is_contig = (t->size == t->extent && t->runs.size() == 1 && t->runs[0].disp == t->lb);
    }
    std::vector<int> ints{count};
    ints.insert(ints.end(), blens, blens + count);
    set_contents(t.get(), combiner, ints, std::vector<MPI_Aint>(disps, disps + count),
                 std::vector<MPI_Datatype>(types, types + count));
    *out = register_type(std::move(t));
    return MPI_SUCCESS;
}

// MPID_Type_create_resized (datatype.cpp:1417-1493)
int dtype_resized(MPI_Datatype oldh, int64_t lb, int64_t extent, MPI_Datatype* out)
{
    std::lock_guard<std::recursive_mutex> g(g_mu);
    Dtype* o = lookup_locked(oldh);
    if (!o) { set_error("invalid oldtype 0x%x", oldh); return MPI_ERR_TYPE; }
    auto t = std::make_unique<Dtype>();
    const bool bi = is_builtin_h(oldh);
    t->size = o->size;
    t->sticky_lb = t->sticky_ub = true;
    t->true_lb = bi ? 0 : o->true_lb;
    t->true_ub = bi ? o->size : o->true_ub;
    t->lb = lb;
    t->ub = lb + extent;
    t->extent = extent;
    t->alignsize = bi ? o->size : o->alignsize;
    t->n_elements = bi ? 1 : o->n_elements;
    t->el_size = bi ? o->size : o->el_size;
    t->eltype = bi ? oldh : o->eltype;
    t->is_contig = bi ? (extent == o->size) : (extent == o->size ? o->is_contig : false);
    copy_layout(t.get(), o);
    set_contents(t.get(), 18, {}, {lb, extent}, {oldh});
    *out = register_type(std::move(t));
    return MPI_SUCCESS;
}

// MPID_Type_dup (datatype.cpp:1603-1685): same layout, committed if the old one is
int dtype_dup(MPI_Datatype oldh, MPI_Datatype* out)
{
    std::lock_guard<std::recursive_mutex> g(g_mu);
    Dtype* o = lookup_locked(oldh);
    if (!o) { set_error("invalid oldtype 0x%x", oldh); return MPI_ERR_TYPE; }
    auto t = std::make_unique<Dtype>();
    t->size = o->size; t->lb = o->lb; t->ub = o->ub; t->extent = o->extent;
    t->true_lb = o->true_lb; t->true_ub = o->true_ub;
    t->sticky_lb = o->sticky_lb; t->sticky_ub = o->sticky_ub;
    t->alignsize = o->alignsize; t->eltype = o->eltype; t->el_size = o->el_size;
    t->n_elements = o->n_elements; t->is_contig = o->is_contig;
    copy_layout(t.get(), o);
    t->committed = o->committed;
    set_contents(t.get(), 2, {}, {}, {oldh});
    *out = register_type(std::move(t));
    return MPI_SUCCESS;
}

// MPID_Type_convert_subarray (datatype.cpp:3274-3399): vector/hvector nest,
// then struct {MPI_LB at 0, nest at the start offset, MPI_UB at the full extent}.
int dtype_subarray(int ndims, const int* sizes, const int* subsizes, const int* starts, int order,
                   MPI_Datatype oldh, MPI_Datatype* out)
{
    std::lock_guard<std::recursive_mutex> g(g_mu);
    Dtype* o = lookup_locked(oldh);
    if (!o) { set_error("invalid oldtype 0x%x", oldh); return MPI_ERR_TYPE; }
    const int64_t extent = is_builtin_h(oldh) ? o->size : o->extent;
    MPI_Datatype tmp1 = MPI_DATATYPE_NULL, tmp2;
    int rc;
    int64_t disp1;
    auto release = [&](MPI_Datatype h) {
        MPI_Datatype x = h;
        dtype_free(&x);
    };
    if (order == 57) {   // MPI_ORDER_FORTRAN: dimension 0 fastest
        if (ndims == 1) {
            rc = dtype_contiguous(subsizes[0], oldh, &tmp1);
        } else {
            rc = dtype_vector(subsizes[1], subsizes[0], sizes[0], false, oldh, &tmp1, 4);
            int64_t size = (int64_t)sizes[0] * extent;
            for (int i = 2; rc == MPI_SUCCESS && i < ndims; ++i) {
                size *= sizes[i - 1];
                rc = dtype_vector(subsizes[i], 1, size, true, tmp1, &tmp2, 6);
                release(tmp1);
                tmp1 = tmp2;
            }
        }
        disp1 = starts[0];
        int64_t size = 1;
        for (int i = 1; i < ndims; ++i) {
            size *= sizes[i - 1];
            disp1 += size * starts[i];
        }
    } else {             // MPI_ORDER_C: dimension ndims-1 fastest
        if (ndims == 1) {
            rc = dtype_contiguous(subsizes[0], oldh, &tmp1);
        } else {
            rc = dtype_vector(subsizes[ndims - 2], subsizes[ndims - 1], sizes[ndims - 1], false, oldh, &tmp1, 4);
            int64_t size = (int64_t)sizes[ndims - 1] * extent;
            for (int i = ndims - 3; rc == MPI_SUCCESS && i >= 0; --i) {
                size *= sizes[i + 1];
                rc = dtype_vector(subsizes[i], 1, size, true, tmp1, &tmp2, 6);
                release(tmp1);
                tmp1 = tmp2;
            }
        }
        disp1 = starts[ndims - 1];
        int64_t size = 1;
        for (int i = ndims - 2; i >= 0; --i) {
            size *= sizes[i + 1];
            disp1 += size * starts[i];
        }
    }
    if (rc != MPI_SUCCESS) return rc;
    disp1 *= extent;
    int64_t disp2 = extent;
    for (int i = 0; i < ndims; ++i) disp2 *= sizes[i];
    const int blk[3] = {1, 1, 1};
    const MPI_Aint d[3] = {0, disp1, disp2};
    const MPI_Datatype ty[3] = {MPI_LB, tmp1, MPI_UB};
    rc = dtype_struct(3, blk, d, ty, out, 12);
    release(tmp1);
    if (rc != MPI_SUCCESS) return rc;
    Dtype* t = lookup_locked(*out);
    for (MPI_Datatype h : t->types)
        if (dtype_is_derived(h)) { MPI_Datatype x = h; dtype_free(&x); }
    std::vector<int> ints{ndims};
    ints.insert(ints.end(), sizes, sizes + ndims);
    ints.insert(ints.end(), subsizes, subsizes + ndims);
    ints.insert(ints.end(), starts, starts + ndims);
    ints.push_back(order);
    set_contents(t, 13, ints, {}, {oldh});
    if (dtype_is_derived(oldh)) o->refs++;
    return MPI_SUCCESS;
}

// ---- MPI_Type_create_darray (api/mpi_datatype.cpp:218-600) ------------------
namespace {

constexpr int kDistBlock = 121, kDistCyclic = 122, kDfltDarg = -49767;

void free_tmp(MPI_Datatype h)
{
    MPI_Datatype x = h;
    if (dtype_is_derived(x)) dtype_free(&x);
}

// MPIR_Type_block (mpid/datatype.cpp:409-509)
int darray_block(const int* gsizes, int dim, int ndims, int nprocs, int rank, int darg, int order,
                 int64_t orig_extent, MPI_Datatype old, MPI_Datatype* out, int64_t* st_offset)
{
    const int global_size = gsizes[dim];
    int blksize;
    if (darg == kDfltDarg) {
        blksize = (global_size + nprocs - 1) / nprocs;
    } else {
        blksize = darg;
        if (blksize <= 0) { set_error("darray block size %d", blksize); return MPI_ERR_ARG; }
        if ((int64_t)blksize * nprocs < global_size) {
            set_error("darray blocks of %d x %d processes do not cover %d", blksize, nprocs, global_size);
            return MPI_ERR_ARG;
        }
    }
    const int64_t j = global_size - (int64_t)blksize * rank;
    const int mysize = (int)std::max<int64_t>(0, std::min<int64_t>(blksize, j));
    const bool fastest = order == MPI_ORDER_FORTRAN ? dim == 0 : dim == ndims - 1;
    int rc;
    if (fastest) {
        rc = dtype_contiguous(mysize, old, out);
    } else {
        int64_t stride = orig_extent;
        if (order == MPI_ORDER_FORTRAN)
            for (int i = 0; i < dim; ++i) stride *= gsizes[i];
        else
            for (int i = ndims - 1; i > dim; --i) stride *= gsizes[i];
        rc = dtype_vector(mysize, 1, stride, true, old, out, 6);
    }
    if (rc != MPI_SUCCESS) return rc;
    *st_offset = mysize == 0 ? 0 : (int64_t)blksize * rank;
    return MPI_SUCCESS;
}

// MPIR_Type_cyclic (mpid/datatype.cpp:512-637)
int darray_cyclic(const int* gsizes, int dim, int ndims, int nprocs, int rank, int darg, int order,
                  int64_t orig_extent, MPI_Datatype old, MPI_Datatype* out, int64_t* st_offset)
{
    const int blksize = darg == kDfltDarg ? 1 : darg;
    if (blksize <= 0) { set_error("darray cyclic block size %d", blksize); return MPI_ERR_ARG; }
    const int64_t st_index = (int64_t)rank * blksize, end_index = gsizes[dim] - 1;
    int64_t local_size = 0;
    if (end_index >= st_index) {
        const int64_t per = (int64_t)nprocs * blksize;
        local_size = ((end_index - st_index + 1) / per) * blksize;
        local_size += std::min<int64_t>((end_index - st_index + 1) % per, blksize);
    }
    const int count = (int)(local_size / blksize), rem = (int)(local_size % blksize);
    int64_t stride = (int64_t)nprocs * blksize * orig_extent;
    if (order == MPI_ORDER_FORTRAN)
        for (int i = 0; i < dim; ++i) stride *= gsizes[i];
    else
        for (int i = ndims - 1; i > dim; --i) stride *= gsizes[i];
    MPI_Datatype t;
    int rc = dtype_vector(count, blksize, stride, true, old, &t, 6);
    if (rc != MPI_SUCCESS) return rc;
    if (rem) {
        // the last, short block is appended as a struct member
        const int blk[2] = {1, rem};
        const MPI_Aint d[2] = {0, (MPI_Aint)count * stride};
        const MPI_Datatype ty[2] = {t, old};
        MPI_Datatype tmp;
        rc = dtype_struct(2, blk, d, ty, &tmp, 12);
        free_tmp(t);
        if (rc != MPI_SUCCESS) return rc;
        t = tmp;
    }
    const bool first = order == MPI_ORDER_FORTRAN ? dim == 0 : dim == ndims - 1;
    if (first) {
        // the first dimension's offset and extent are set with LB / UB markers
        const int blk[3] = {1, 1, 1};
        const MPI_Aint d[3] = {0, (MPI_Aint)rank * blksize * orig_extent, orig_extent * gsizes[dim]};
        const MPI_Datatype ty[3] = {MPI_LB, t, MPI_UB};
        MPI_Datatype tmp;
        rc = dtype_struct(3, blk, d, ty, &tmp, 12);
        free_tmp(t);
        if (rc != MPI_SUCCESS) return rc;
        t = tmp;
        *st_offset = 0;
    } else {
        *st_offset = (int64_t)rank * blksize;
    }
    if (local_size == 0) *st_offset = 0;
    *out = t;
    return MPI_SUCCESS;
}

}  // namespace

int dtype_darray(int size, int rank, int ndims, const int* gsizes, const int* distribs, const int* dargs,
                 const int* psizes, int order, MPI_Datatype oldh, MPI_Datatype* out)
{
    std::lock_guard<std::recursive_mutex> g(g_mu);
    Dtype* o = lookup_locked(oldh);
    if (!o) { set_error("invalid oldtype 0x%x", oldh); return MPI_ERR_TYPE; }
    const int64_t orig_extent = is_builtin_h(oldh) ? o->size : o->extent;
    // position in the process grid, row-major (api/mpi_datatype.cpp:346-353)
    std::vector<int> coords((size_t)std::max(ndims, 1));
    int procs = size, tmp_rank = rank;
    for (int i = 0; i < ndims; ++i) {
        if (psizes[i] == 0 || procs / psizes[i] == 0) {
            // the reference divides by zero here
            set_error("darray process grid does not divide size %d", size);
            return MPI_ERR_ARG;
        }
        procs /= psizes[i];
        coords[(size_t)i] = tmp_rank / procs;
        tmp_rank %= procs;
    }
    std::vector<int64_t> st((size_t)std::max(ndims, 1), 0);
    MPI_Datatype cur = oldh;
    auto step = [&](int i) -> int {
        MPI_Datatype nt;
        int rc;
        if (distribs[i] == kDistCyclic)
            rc = darray_cyclic(gsizes, i, ndims, psizes[i], coords[(size_t)i], dargs[i], order, orig_extent, cur,
                               &nt, &st[(size_t)i]);
        else if (distribs[i] == kDistBlock)
            rc = darray_block(gsizes, i, ndims, psizes[i], coords[(size_t)i], dargs[i], order, orig_extent, cur,
                              &nt, &st[(size_t)i]);
        else   // MPI_DISTRIBUTE_NONE: a block distribution over one process
            rc = darray_block(gsizes, i, ndims, psizes[i], coords[(size_t)i], kDfltDarg, order, orig_extent, cur,
                              &nt, &st[(size_t)i]);
        if (cur != oldh) free_tmp(cur);
        cur = rc == MPI_SUCCESS ? nt : oldh;
        return rc;
    };
    int64_t disp1 = 0, tmp_size = 1;
    int rc = MPI_SUCCESS;
    if (order == MPI_ORDER_FORTRAN) {
        for (int i = 0; rc == MPI_SUCCESS && i < ndims; ++i) rc = step(i);
        if (ndims > 0) disp1 = st[0];
        for (int i = 1; i < ndims; ++i) {
            tmp_size *= gsizes[i - 1];
            disp1 += tmp_size * st[(size_t)i];
        }
    } else {
        for (int i = ndims - 1; rc == MPI_SUCCESS && i >= 0; --i) rc = step(i);
        if (ndims > 0) disp1 = st[(size_t)ndims - 1];
        for (int i = ndims - 2; i >= 0; --i) {
            tmp_size *= gsizes[i + 1];
            disp1 += tmp_size * st[(size_t)i];
        }
    }
    if (rc != MPI_SUCCESS) return rc;
    disp1 *= orig_extent;
    int64_t disp2 = orig_extent;
    for (int i = 0; i < ndims; ++i) disp2 *= gsizes[i];
    const int blk[3] = {1, 1, 1};
    const MPI_Aint d[3] = {0, disp1, disp2};
    const MPI_Datatype ty[3] = {MPI_LB, cur, MPI_UB};
    rc = dtype_struct(3, blk, d, ty, out, 12);
    if (cur != oldh) free_tmp(cur);
    if (rc != MPI_SUCCESS) return rc;
    Dtype* t = lookup_locked(*out);
    for (MPI_Datatype h : t->types) free_tmp(h);      // drop the struct's references
    std::vector<int> ints{size, rank, ndims};
    ints.insert(ints.end(), gsizes, gsizes + ndims);
    ints.insert(ints.end(), distribs, distribs + ndims);
    ints.insert(ints.end(), dargs, dargs + ndims);
    ints.insert(ints.end(), psizes, psizes + ndims);
    ints.push_back(order);
    set_contents(t, 14, ints, {}, {oldh});
    if (dtype_is_derived(oldh)) o->refs++;
    return MPI_SUCCESS;
}

int dtype_commit(MPI_Datatype h)
{
    std::lock_guard<std::recursive_mutex> g(g_mu);
    Dtype* t = lookup_locked(h);
    if (!t) return MPI_ERR_TYPE;
    t->committed = true;
    return MPI_SUCCESS;
}

int dtype_free(MPI_Datatype* h)
{
    std::lock_guard<std::recursive_mutex> g(g_mu);
    if (!dtype_is_derived(*h)) return MPI_ERR_TYPE;
    const size_t idx = (unsigned)*h & 0x03ffffffu;
    if (idx >= g_slots.size() || !g_slots[idx]) return MPI_ERR_TYPE;
    Dtype* t = g_slots[idx];
    if (--t->refs <= 0) {
        std::vector<MPI_Datatype> held = t->types;
        g_slots[idx] = nullptr;
        destroy(t);
        for (MPI_Datatype x : held)
            if (dtype_is_derived(x)) { MPI_Datatype y = x; dtype_free(&y); }
    }
    *h = MPI_DATATYPE_NULL;
    return MPI_SUCCESS;
}

// ---------------------------------------------------------------------------
// device layout
// ---------------------------------------------------------------------------
namespace {

int build_dev_layout(Dtype* t)
{
    if (t->dev_ready) return MPI_SUCCESS;
    DevLayout L;
    L.size = t->size;
    L.extent = t->extent;
    L.nruns = dtype_nruns(t);
    int64_t al = 16;
    al = std::min(al, lowbit_align(t->size));
    al = std::min(al, lowbit_align(t->extent));
    if (t->rn) {
        // compact regular form: no run table at all
        al = std::min({al, lowbit_align(t->rfirst), lowbit_align(t->rlen), lowbit_align(t->rstride)});
        if (t->rn2 > 1) al = std::min(al, lowbit_align(t->rstride2));
        L.align = (int)al;
        L.regular = 1;
        L.first = t->rfirst;
        L.blen = t->rlen;
        L.stride = t->rstride;
        if (t->rn2 > 1) {
            L.n1 = t->rn;
            L.stride2 = t->rstride2;
        }
        t->dev = L;
        t->dev_ready = true;
        return MPI_SUCCESS;
    }
    for (const DtRun& r : t->runs) {
        al = std::min(al, lowbit_align(r.disp));
        al = std::min(al, lowbit_align(r.len));
    }
    L.align = (int)al;
    const size_t n = t->runs.size();
    bool regular = n >= 1;
    const int64_t stride0 = n > 1 ? t->runs[1].disp - t->runs[0].disp : 0;
    for (size_t k = 1; regular && k < n; ++k)
        regular = t->runs[k].len == t->runs[0].len && t->runs[k].disp - t->runs[k - 1].disp == stride0;
    if (regular) {
        L.regular = 1;
        L.first = t->runs[0].disp;
        L.blen = t->runs[0].len;
        L.stride = n > 1 ? t->runs[1].disp - t->runs[0].disp : t->runs[0].len;
    } else {
        int rc = ensure_device();
        if (rc != MPI_SUCCESS) return rc;
        std::vector<int64_t> host(2 * n + 1);
        int64_t acc = 0;
        for (size_t k = 0; k < n; ++k) {
            host[k] = t->runs[k].disp;
            host[n + k] = acc;
            acc += t->runs[k].len;
        }
        host[2 * n] = acc;
        void* mem = nullptr;
        hipError_t e = hipMalloc(&mem, host.size() * sizeof(int64_t));
        if (e != hipSuccess) return hip_fail(e, "datatype layout allocation");
        if ((rc = xfer_sync(mem, host.data(), host.size() * sizeof(int64_t), internal_stream())) != MPI_SUCCESS) {
            (void)hipFree(mem);
            return rc;
        }
        t->dev_mem = mem;
        L.disp = static_cast<const int64_t*>(mem);
        L.poff = static_cast<const int64_t*>(mem) + n;
    }
    t->dev = L;
    t->dev_ready = true;
    return MPI_SUCCESS;
}

int64_t ptr_align(const void* p) { return lowbit_align((int64_t)(uintptr_t)p); }

// Device scratch for staging host operands (grows; guarded by its own lock).
std::mutex g_stage_mu;
void* g_stage = nullptr;
size_t g_stage_bytes = 0;

void* stage_buffer(size_t bytes)
{
    if (bytes <= g_stage_bytes) return g_stage;
    if (g_stage) (void)hipFree(g_stage);
    g_stage = nullptr;
    g_stage_bytes = 0;
    if (hipMalloc(&g_stage, bytes) != hipSuccess) {
        g_stage = nullptr;
        return nullptr;
    }
    g_stage_bytes = bytes;
    return g_stage;
}

}  // namespace

void dtype_serialize(const Dtype* t, std::vector<int64_t>& out)
{
    out.push_back(t->size);
    out.push_back(t->extent);
    out.push_back((int64_t)t->eltype);
    if (t->rn && t->rn2 > 1) {   // two-level compact form: flag -2, then first, len, stride, n, stride2, n2
        out.insert(out.end(), {-2, t->rfirst, t->rlen, t->rstride, t->rn, t->rstride2, t->rn2});
        return;
    }
    if (t->rn) {            // compact form: flag -1, then first, len, stride, n
        out.insert(out.end(), {-1, t->rfirst, t->rlen, t->rstride, t->rn});
        return;
    }
    out.push_back((int64_t)t->runs.size());
    for (const DtRun& r : t->runs) {
        out.push_back(r.disp);
        out.push_back(r.len);
    }
}

Dtype* dtype_from_blob(const int64_t* b, int64_t avail)
{
    if (avail >= 10 && b[3] == -2) {
        const int64_t lim = (int64_t)1 << 40;
        // every product bounded before it is formed (the blob comes from
        // another process): b[7] * b[9] <= 2^40, then rlen <= 2^62 / that
        if (b[5] <= 0 || b[7] <= 0 || b[9] <= 1 || b[7] > lim || b[9] > lim / b[7] ||
            b[5] > ((int64_t)1 << 62) / (b[7] * b[9]) || b[7] * b[9] * b[5] != b[0])
            return nullptr;
        auto* t = new Dtype();
        t->size = b[0];
        t->extent = b[1];
        t->eltype = (MPI_Datatype)b[2];
        const TypeInfo* ti = type_info(t->eltype);
        t->el_size = ti ? ti->size : -1;
        t->committed = true;
        t->rfirst = b[4];
        t->rlen = b[5];
        t->rstride = b[6];
        t->rn = b[7];
        t->rstride2 = b[8];
        t->rn2 = b[9];
        return t;
    }
    if (avail >= 8 && b[3] == -1) {
        if (b[7] <= 0 || b[5] <= 0 || b[7] > ((int64_t)1 << 40) || b[5] > ((int64_t)1 << 62) / b[7] ||
            b[7] * b[5] != b[0])
            return nullptr;
        auto* t = new Dtype();
        t->size = b[0];
        t->extent = b[1];
        t->eltype = (MPI_Datatype)b[2];
        const TypeInfo* ti = type_info(t->eltype);
        t->el_size = ti ? ti->size : -1;
        t->committed = true;
        t->rfirst = b[4];
        t->rlen = b[5];
        t->rstride = b[6];
        t->rn = b[7];
        return t;
    }
    if (avail < 4 || b[3] < 0 || b[3] > kMaxRuns || avail < 4 + 2 * b[3]) return nullptr;
    auto* t = new Dtype();
    t->size = b[0];
    t->extent = b[1];
    t->eltype = (MPI_Datatype)b[2];
    const TypeInfo* ti = type_info(t->eltype);
    t->el_size = ti ? ti->size : -1;
    t->committed = true;
    t->runs.resize((size_t)b[3]);
    int64_t sum = 0;
    for (int64_t k = 0; k < b[3]; ++k) {
        t->runs[(size_t)k] = {b[4 + 2 * k], b[5 + 2 * k]};
        sum += b[5 + 2 * k];
    }
    if (sum != t->size) {
        delete t;
        return nullptr;
    }
    return t;
}

void dtype_delete(Dtype* t)
{
    if (t) destroy(t);
}

void dt_span(const Dtype* t, int64_t count, int64_t* lo, int64_t* hi)
{
    if ((t->runs.empty() && !t->rn) || count <= 0) { *lo = *hi = 0; return; }
    int64_t rl = INT64_MAX, rh = INT64_MIN;
    if (t->rn) {
        const int64_t d1 = (t->rn - 1) * t->rstride, d2 = (t->rn2 - 1) * t->rstride2;
        rl = t->rfirst + std::min<int64_t>(0, d1) + std::min<int64_t>(0, d2);
        rh = t->rfirst + std::max<int64_t>(0, d1) + std::max<int64_t>(0, d2) + t->rlen;
    }
    for (const DtRun& r : t->runs) {
        rl = std::min(rl, r.disp);
        rh = std::max(rh, r.disp + r.len);
    }
    const int64_t shift = (count - 1) * t->extent;
    *lo = rl + std::min<int64_t>(0, shift);
    *hi = rh + std::max<int64_t>(0, shift);
}

int dt_pack_dev(const Dtype* tc, int64_t count, const void* typed, void* packed, hipStream_t s)
{
    if (count <= 0 || tc->size == 0) return MPI_SUCCESS;
    Dtype* t = const_cast<Dtype*>(tc);
    int rc;
    {
        std::lock_guard<std::recursive_mutex> g(g_mu);
        rc = build_dev_layout(t);
    }
    if (rc != MPI_SUCCESS) return rc;
    DevLayout L = t->dev;
    L.align = (int)std::min<int64_t>({(int64_t)L.align, ptr_align(typed), ptr_align(packed)});
    hipError_t e = launch_dt_copy(L, count, const_cast<void*>(typed), packed, false, s);
    return e == hipSuccess ? MPI_SUCCESS : hip_fail(e, "datatype pack");
}

int dt_unpack_dev(const Dtype* tc, int64_t count, const void* packed, void* typed, hipStream_t s)
{
    if (count <= 0 || tc->size == 0) return MPI_SUCCESS;
    Dtype* t = const_cast<Dtype*>(tc);
    int rc;
    {
        std::lock_guard<std::recursive_mutex> g(g_mu);
        rc = build_dev_layout(t);
    }
    if (rc != MPI_SUCCESS) return rc;
    DevLayout L = t->dev;
    L.align = (int)std::min<int64_t>({(int64_t)L.align, ptr_align(typed), ptr_align(packed)});
    hipError_t e = launch_dt_copy(L, count, typed, const_cast<void*>(packed), true, s);
    return e == hipSuccess ? MPI_SUCCESS : hip_fail(e, "datatype unpack");
}

int dt_acc_dev(int opidx, const Dtype* tc, int64_t count, const void* packed, void* typed, hipStream_t s)
{
    if (count <= 0 || tc->size == 0 || opidx == O_NOOP) return MPI_SUCCESS;
    if (opidx == O_REPLACE) return dt_unpack_dev(tc, count, packed, typed, s);
    // the reference applies the op with dtp->eltype (packethandling.cpp:2993-3001):
    // a mixed type (eltype NULL) or an illegal pair only sets op_errno
    const TypeInfo* ti = type_info(tc->eltype);
    if (!ti || op_check_dtype(opidx, tc->eltype) != MPI_SUCCESS) return MPI_SUCCESS;
    // every run holds whole elements (true for any type built from one basic type)
    if (tc->rn && tc->rlen % ti->size) {
        set_error("datatype runs split elements of 0x%x", tc->eltype);
        return MPI_ERR_TYPE;
    }
    for (const DtRun& r : tc->runs)
        if (r.len % ti->size) {
            set_error("datatype runs split elements of 0x%x", tc->eltype);
            return MPI_ERR_TYPE;
        }
    Dtype* t = const_cast<Dtype*>(tc);
    int rc;
    {
        std::lock_guard<std::recursive_mutex> g(g_mu);
        rc = build_dev_layout(t);
    }
    if (rc != MPI_SUCCESS) return rc;
    DevLayout L = t->dev;
    L.align = (int)std::min<int64_t>({(int64_t)L.align, ptr_align(typed), ptr_align(packed)});
    hipError_t e = launch_dt_acc(opidx, ti->kind, L, count, packed, typed, s);
    return e == hipSuccess ? MPI_SUCCESS : hip_fail(e, "datatype accumulate");
}

int dt_pack_any(const Dtype* t, int64_t count, const void* typed, void* packed)
{
    if (count <= 0 || t->size == 0) return MPI_SUCCESS;
    int rc = ensure_device();
    if (rc != MPI_SUCCESS) return rc;
    hipStream_t s = internal_stream();
    const size_t pbytes = (size_t)(count * t->size);
    int64_t lo, hi;
    dt_span(t, count, &lo, &hi);
    const BufInfo bt = classify(static_cast<const char*>(typed) + lo);
    const BufInfo bp = classify(packed);
    std::lock_guard<std::mutex> g(g_stage_mu);
    const char* tdev = static_cast<const char*>(typed);
    char* pdev = static_cast<char*>(packed);
    const size_t span = (size_t)(hi - lo);
    const bool stage_t = bt.place != Place::Device, stage_p = bp.place != Place::Device;
    char* st = static_cast<char*>(stage_buffer((stage_t ? span + 16 : 0) + (stage_p ? pbytes + 16 : 0)));
    if ((stage_t || stage_p) && !st) { set_error("datatype staging allocation failed"); return MPI_ERR_NO_MEM; }
    hipError_t e = hipSuccess;
    if (stage_t) {
        // keep the user's address modulo 16 so the kernel's granule choice holds
        const uintptr_t mis = (uintptr_t)(static_cast<const char*>(typed) + lo) & 15;
        char* base = st + mis;
        if ((rc = xfer_sync(base, static_cast<const char*>(typed) + lo, span, s)) != MPI_SUCCESS) return rc;
        tdev = base - lo;
        st += span + 16;
    } else {
        tdev = static_cast<const char*>(bt.dev) - lo;
    }
    if (stage_p) pdev = st + ((uintptr_t)packed & 15);
    else pdev = static_cast<char*>(bp.dev);
    if (e != hipSuccess) return hip_fail(e, "datatype pack staging");
    rc = dt_pack_dev(t, count, tdev, pdev, s);
    if (rc == MPI_SUCCESS && stage_p) return xfer_sync(packed, pdev, pbytes, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    return rc != MPI_SUCCESS ? rc : (e == hipSuccess ? MPI_SUCCESS : hip_fail(e, "datatype pack"));
}

int dt_unpack_any(const Dtype* t, int64_t count, const void* packed, void* typed)
{
    if (count <= 0 || t->size == 0) return MPI_SUCCESS;
    int rc = ensure_device();
    if (rc != MPI_SUCCESS) return rc;
    hipStream_t s = internal_stream();
    const size_t pbytes = (size_t)(count * t->size);
    int64_t lo, hi;
    dt_span(t, count, &lo, &hi);
    const BufInfo bt = classify(static_cast<char*>(typed) + lo);
    const BufInfo bp = classify(packed);
    std::lock_guard<std::mutex> g(g_stage_mu);
    const size_t span = (size_t)(hi - lo);
    const bool stage_t = bt.place != Place::Device, stage_p = bp.place != Place::Device;
    char* st = static_cast<char*>(stage_buffer((stage_t ? span + 16 : 0) + (stage_p ? pbytes + 16 : 0)));
    if ((stage_t || stage_p) && !st) { set_error("datatype staging allocation failed"); return MPI_ERR_NO_MEM; }
    hipError_t e = hipSuccess;
    char* tdev;
    const char* pdev;
    char* user_lo = static_cast<char*>(typed) + lo;
    char* tbase = nullptr;
    if (stage_t) {
        // the gaps between runs must keep the caller's bytes: stage the whole
        // span in, unpack into it, copy it back
        tbase = st + ((uintptr_t)user_lo & 15);
        if ((rc = xfer_sync(tbase, user_lo, span, s)) != MPI_SUCCESS) return rc;
        tdev = tbase - lo;
        st += span + 16;
    } else {
        tdev = static_cast<char*>(bt.dev) - lo;
    }
    if (e == hipSuccess && stage_p) {
        char* pb = st + ((uintptr_t)packed & 15);
        if ((rc = xfer_sync(pb, packed, pbytes, s)) != MPI_SUCCESS) return rc;
        pdev = pb;
    } else {
        pdev = static_cast<const char*>(bp.dev);
    }
    if (e != hipSuccess) return hip_fail(e, "datatype unpack staging");
    rc = dt_unpack_dev(t, count, pdev, tdev, s);
    if (rc == MPI_SUCCESS && stage_t) return xfer_sync(user_lo, tbase, span, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    return rc != MPI_SUCCESS ? rc : (e == hipSuccess ? MPI_SUCCESS : hip_fail(e, "datatype unpack"));
}

int dt_copy_any(const void* src, int64_t scount, MPI_Datatype sdt, void* dst, int64_t rcount, MPI_Datatype rdt)
{
    Dtype* st = dtype_lookup(sdt);
    Dtype* rt = dtype_lookup(rdt);
    if (!st || !rt) { set_error("invalid datatype"); return MPI_ERR_TYPE; }
    const int64_t sbytes = scount * st->size, rbytes = rcount * rt->size;
    int64_t n = std::min(sbytes, rbytes);
    DtRun s1{0, 0}, r1{0, 0};
    const bool s_contig = single_run(st, &s1) && (scount <= 1 || st->size == st->extent);
    const bool r_contig = single_run(rt, &r1) && (rcount <= 1 || rt->size == rt->extent);
    int rc = MPI_SUCCESS;
    if (n > 0) {
        if (s_contig && r_contig) {
            rc = copy_any(static_cast<char*>(dst) + r1.disp, static_cast<const char*>(src) + s1.disp, (size_t)n);
        } else if (sbytes == rbytes) {
            // pack the source into a device buffer, unpack it into the target
            rc = ensure_device();
            void* tmp = nullptr;
            if (rc == MPI_SUCCESS && hipMalloc(&tmp, (size_t)n) != hipSuccess) rc = MPI_ERR_NO_MEM;
            if (rc == MPI_SUCCESS) rc = dt_pack_any(st, scount, src, tmp);
            if (rc == MPI_SUCCESS) rc = dt_unpack_any(rt, rcount, tmp, dst);
            if (tmp) (void)hipFree(tmp);
        } else {
            set_error("datatype copy of %lld bytes into %lld (partial derived copies unsupported)",
                      (long long)sbytes, (long long)rbytes);
            rc = MPI_ERR_TYPE;
        }
    }
    if (rc == MPI_SUCCESS && sbytes > rbytes) {
        set_error("message truncated: %lld bytes into %lld", (long long)sbytes, (long long)rbytes);
        rc = MPI_ERR_TRUNCATE;
    }
    return rc;
}

}  // namespace msx
