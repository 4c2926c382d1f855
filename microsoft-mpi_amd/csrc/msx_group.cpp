// msx_group.cpp — MPI groups: ordered lists of process ids (MPI_COMM_WORLD
// ranks), the argument of the PSCW synchronisation (MPI_Win_post / start).
//
// Reference: api/mpi_group.cpp (cited per function), MPIR_Group_check_valid_ranks
// / _ranges (mpid/group.cpp:249-380), MPI_Comm_group (api/mpi_comm.cpp:677).
// Handles: MPI_GROUP_EMPTY = 0x48000000 is direct index 0 of kind GROUP; the
// groups this library creates are 0x48000000 | index, index >= 1.  Argument
// checks keep the reference's order; errors go through MPI_COMM_WORLD's handler
// (MPIR_Err_return_comm(NULL, ...)).  Host-only: no GPU is involved.
#include <algorithm>
#include <mutex>
#include <set>
#include <vector>

#include "../../include/mpi.h"
#include "msx_comm.h"
#include "msx_dtype.h"
#include "msx_runtime.h"

using namespace msx;

#define MSX_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

constexpr unsigned kGroupDirect = 0x48000000u;

struct GroupObj {
    std::vector<int> lpid;
};

std::mutex g_mu;
std::vector<GroupObj*> g_groups(1, nullptr);      // index 0: MPI_GROUP_EMPTY (no object)

int fail(const char* fn, int code) { return api_err_return(fn, code); }

// MpiaGroupValidateHandle
int lookup(MPI_Group h, std::vector<int>* out)
{
    if (h == MPI_GROUP_NULL) { set_error("null group"); return MPI_ERR_GROUP; }
    if (((unsigned)h & 0xfc000000u) != kGroupDirect) { set_error("invalid group 0x%x", (unsigned)h); return MPI_ERR_GROUP; }
    const size_t idx = (unsigned)h & 0x03ffffffu;
    std::lock_guard<std::mutex> g(g_mu);
    if (idx == 0) { out->clear(); return MPI_SUCCESS; }
    if (idx >= g_groups.size() || !g_groups[idx]) { set_error("invalid group 0x%x", (unsigned)h); return MPI_ERR_GROUP; }
    *out = g_groups[idx]->lpid;
    return MPI_SUCCESS;
}

// this process's id: its MPI_COMM_WORLD rank
int my_lpid()
{
    Comm* w = world();
    return w ? w->rank : 0;
}

int rank_in(const std::vector<int>& lpid, int id)
{
    for (size_t i = 0; i < lpid.size(); ++i)
        if (lpid[i] == id) return (int)i;
    return MPI_UNDEFINED;
}

// MPIR_Group_check_valid_ranks (mpid/group.cpp:249-289)
int check_ranks(size_t size, const int ranks[], int n)
{
    if (n < 0 || (size_t)n > size) {
        set_error("**rankarraysize %d %zu", n, size);
        return MPI_ERR_ARG;
    }
    std::vector<int> seen(size, 0);
    for (int i = 0; i < n; ++i) {
        if (ranks[i] < 0 || (size_t)ranks[i] >= size) {
            set_error("**rankarray %d %d %zu", i, ranks[i], size - 1);
            return MPI_ERR_RANK;
        }
        if (seen[(size_t)ranks[i]]) {
            set_error("**rankdup %d %d %d", i, ranks[i], seen[(size_t)ranks[i]] - 1);
            return MPI_ERR_RANK;
        }
        seen[(size_t)ranks[i]] = i + 1;
    }
    return MPI_SUCCESS;
}

// MPIR_Group_check_valid_ranges (mpid/group.cpp:299-380); fills the ranks the
// ranges name, in range order
int check_ranges(size_t size, const int ranges[][3], int n, std::vector<int>* named)
{
    if (n < 0 || (size_t)n > size) {
        set_error("**rangessize %d %zu", n, size);
        return MPI_ERR_ARG;
    }
    std::vector<int> seen(size, 0);
    named->clear();
    for (int i = 0; i < n; ++i) {
        const int first = ranges[i][0], last = ranges[i][1], stride = ranges[i][2];
        if (first < 0 || (size_t)first >= size) {
            set_error("**rangestartinvalid %d %d %zu", i, first, size);
            return MPI_ERR_ARG;
        }
        if (stride == 0) { set_error("**stridezero"); return MPI_ERR_ARG; }
        const int act_last = first + stride * ((last - first) / stride);
        if (last < 0 || (size_t)act_last >= size) {
            set_error("**rangeendinvalid %d %d %zu", i, last, size);
            return MPI_ERR_ARG;
        }
        if ((stride > 0 && first > last) || (stride < 0 && first < last)) {
            set_error("**stride %d %d %d", first, last, stride);
            return MPI_ERR_ARG;
        }
        for (int j = first; stride > 0 ? j <= last : j >= last; j += stride) {
            if (seen[(size_t)j]) {
                set_error("**rangedup %d %d %d", j, i, seen[(size_t)j] - 1);
                return MPI_ERR_ARG;
            }
            seen[(size_t)j] = i + 1;
            named->push_back(j);
        }
    }
    return MPI_SUCCESS;
}

}  // namespace

namespace msx {

int group_members(MPI_Group g, std::vector<int>* lpid) { return lookup(g, lpid); }

int group_create(const std::vector<int>& lpid, MPI_Group* out)
{
    if (lpid.empty()) {
        *out = MPI_GROUP_EMPTY;
        return MPI_SUCCESS;
    }
    auto* g = new GroupObj{lpid};
    std::lock_guard<std::mutex> lk(g_mu);
    size_t idx = 1;
    while (idx < g_groups.size() && g_groups[idx]) ++idx;
    if (idx == g_groups.size()) g_groups.push_back(nullptr);
    g_groups[idx] = g;
    *out = (MPI_Group)(kGroupDirect | (unsigned)idx);
    return MPI_SUCCESS;
}

}  // namespace msx

// api/mpi_comm.cpp:677-730
MSX_EXPORT int MPI_Comm_group(MPI_Comm comm, MPI_Group* group)
{
    api_require_init("MPI_Comm_group");
    Comm* c = comm == MPI_COMM_NULL ? nullptr : lookup_comm(comm);
    if (!c) { set_error("invalid communicator 0x%x", (unsigned)comm); return fail("MPI_Comm_group", MPI_ERR_COMM); }
    if (!group) { set_error("null group"); return fail("MPI_Comm_group", MPI_ERR_ARG); }
    return fail("MPI_Comm_group", group_create(c->lpid, group));
}

// api/mpi_group.cpp:1216-1260
MSX_EXPORT int MPI_Group_size(MPI_Group group, int* size)
{
    api_require_init("MPI_Group_size");
    std::vector<int> m;
    int rc = lookup(group, &m);
    if (rc == MPI_SUCCESS && !size) { set_error("null size"); rc = MPI_ERR_ARG; }
    if (rc == MPI_SUCCESS) *size = (int)m.size();
    return fail("MPI_Group_size", rc);
}

// api/mpi_group.cpp:1150-1195: MPI_UNDEFINED when the caller is not a member
MSX_EXPORT int MPI_Group_rank(MPI_Group group, int* rank)
{
    api_require_init("MPI_Group_rank");
    std::vector<int> m;
    int rc = lookup(group, &m);
    if (rc == MPI_SUCCESS && !rank) { set_error("null rank"); rc = MPI_ERR_ARG; }
    if (rc == MPI_SUCCESS) *rank = rank_in(m, my_lpid());
    return fail("MPI_Group_rank", rc);
}

// api/mpi_group.cpp:458-510: MPI_GROUP_EMPTY is never freed
MSX_EXPORT int MPI_Group_free(MPI_Group* group)
{
    api_require_init("MPI_Group_free");
    if (!group) { set_error("null group"); return fail("MPI_Group_free", MPI_ERR_ARG); }
    std::vector<int> m;
    int rc = lookup(*group, &m);
    if (rc != MPI_SUCCESS) return fail("MPI_Group_free", rc);
    if (*group != MPI_GROUP_EMPTY) {
        std::lock_guard<std::mutex> g(g_mu);
        const size_t idx = (unsigned)*group & 0x03ffffffu;
        delete g_groups[idx];
        g_groups[idx] = nullptr;
    }
    *group = MPI_GROUP_NULL;
    return MPI_SUCCESS;
}

// api/mpi_group.cpp:543-635
MSX_EXPORT int MPI_Group_incl(MPI_Group group, int n, const int ranks[], MPI_Group* newgroup)
{
    api_require_init("MPI_Group_incl");
    std::vector<int> m;
    int rc = lookup(group, &m);
    if (rc == MPI_SUCCESS && n < 0) { set_error("**argneg n %d", n); rc = MPI_ERR_ARG; }
    if (rc == MPI_SUCCESS && n > 0 && !ranks) { set_error("null ranks"); rc = MPI_ERR_ARG; }
    if (rc == MPI_SUCCESS && !newgroup) { set_error("null newgroup"); rc = MPI_ERR_ARG; }
    if (rc == MPI_SUCCESS) rc = check_ranks(m.size(), ranks, n);
    if (rc != MPI_SUCCESS) return fail("MPI_Group_incl", rc);
    std::vector<int> out;
    for (int i = 0; i < n; ++i) out.push_back(m[(size_t)ranks[i]]);
    return fail("MPI_Group_incl", group_create(out, newgroup));
}

// api/mpi_group.cpp:326-435: the members not listed, in their order
MSX_EXPORT int MPI_Group_excl(MPI_Group group, int n, const int ranks[], MPI_Group* newgroup)
{
    api_require_init("MPI_Group_excl");
    std::vector<int> m;
    int rc = lookup(group, &m);
    if (rc == MPI_SUCCESS && n < 0) { set_error("**argneg n %d", n); rc = MPI_ERR_ARG; }
    if (rc == MPI_SUCCESS && n > 0 && !ranks) { set_error("null ranks"); rc = MPI_ERR_ARG; }
    if (rc == MPI_SUCCESS && !newgroup) { set_error("null newgroup"); rc = MPI_ERR_ARG; }
    if (rc == MPI_SUCCESS) rc = check_ranks(m.size(), ranks, n);
    if (rc != MPI_SUCCESS) return fail("MPI_Group_excl", rc);
    std::vector<char> drop(m.size(), 0);
    for (int i = 0; i < n; ++i) drop[(size_t)ranks[i]] = 1;
    std::vector<int> out;
    for (size_t i = 0; i < m.size(); ++i)
        if (!drop[i]) out.push_back(m[i]);
    return fail("MPI_Group_excl", group_create(out, newgroup));
}

// api/mpi_group.cpp:1001-1125: the ranks the triplets name, in range order
MSX_EXPORT int MPI_Group_range_incl(MPI_Group group, int n, int ranges[][3], MPI_Group* newgroup)
{
    api_require_init("MPI_Group_range_incl");
    std::vector<int> m, named;
    int rc = lookup(group, &m);
    if (rc == MPI_SUCCESS && n > 0 && !ranges) { set_error("null ranges"); rc = MPI_ERR_ARG; }
    if (rc == MPI_SUCCESS && !newgroup) { set_error("null newgroup"); rc = MPI_ERR_ARG; }
    if (rc == MPI_SUCCESS) rc = check_ranges(m.size(), ranges, n, &named);
    if (rc != MPI_SUCCESS) return fail("MPI_Group_range_incl", rc);
    std::vector<int> out;
    for (int r : named) out.push_back(m[(size_t)r]);
    return fail("MPI_Group_range_incl", group_create(out, newgroup));
}

// api/mpi_group.cpp:824-965
MSX_EXPORT int MPI_Group_range_excl(MPI_Group group, int n, int ranges[][3], MPI_Group* newgroup)
{
    api_require_init("MPI_Group_range_excl");
    std::vector<int> m, named;
    int rc = lookup(group, &m);
    if (rc == MPI_SUCCESS && n > 0 && !ranges) { set_error("null ranges"); rc = MPI_ERR_ARG; }
    if (rc == MPI_SUCCESS && !newgroup) { set_error("null newgroup"); rc = MPI_ERR_ARG; }
    if (rc == MPI_SUCCESS) rc = check_ranges(m.size(), ranges, n, &named);
    if (rc != MPI_SUCCESS) return fail("MPI_Group_range_excl", rc);
    std::vector<char> drop(m.size(), 0);
    for (int r : named) drop[(size_t)r] = 1;
    std::vector<int> out;
    for (size_t i = 0; i < m.size(); ++i)
        if (!drop[i]) out.push_back(m[i]);
    return fail("MPI_Group_range_excl", group_create(out, newgroup));
}

namespace {
int two_groups(const char* fn, MPI_Group g1, MPI_Group g2, MPI_Group* newgroup, std::vector<int>* a,
               std::vector<int>* b)
{
    int rc = lookup(g1, a);
    if (rc == MPI_SUCCESS) rc = lookup(g2, b);
    if (rc == MPI_SUCCESS && !newgroup) { set_error("null newgroup"); rc = MPI_ERR_ARG; }
    (void)fn;
    return rc;
}
}  // namespace

// api/mpi_group.cpp:1456-1600: group1's members, then group2's not in group1
MSX_EXPORT int MPI_Group_union(MPI_Group group1, MPI_Group group2, MPI_Group* newgroup)
{
    api_require_init("MPI_Group_union");
    std::vector<int> a, b;
    int rc = two_groups("MPI_Group_union", group1, group2, newgroup, &a, &b);
    if (rc != MPI_SUCCESS) return fail("MPI_Group_union", rc);
    std::set<int> in_a(a.begin(), a.end());
    std::vector<int> out = a;
    for (int x : b)
        if (!in_a.count(x)) out.push_back(x);
    return fail("MPI_Group_union", group_create(out, newgroup));
}

// api/mpi_group.cpp:665-785: group1's members that are in group2, group1's order
MSX_EXPORT int MPI_Group_intersection(MPI_Group group1, MPI_Group group2, MPI_Group* newgroup)
{
    api_require_init("MPI_Group_intersection");
    std::vector<int> a, b;
    int rc = two_groups("MPI_Group_intersection", group1, group2, newgroup, &a, &b);
    if (rc != MPI_SUCCESS) return fail("MPI_Group_intersection", rc);
    std::set<int> in_b(b.begin(), b.end());
    std::vector<int> out;
    for (int x : a)
        if (in_b.count(x)) out.push_back(x);
    return fail("MPI_Group_intersection", group_create(out, newgroup));
}

// api/mpi_group.cpp:166-290: group1's members not in group2, group1's order
MSX_EXPORT int MPI_Group_difference(MPI_Group group1, MPI_Group group2, MPI_Group* newgroup)
{
    api_require_init("MPI_Group_difference");
    std::vector<int> a, b;
    int rc = two_groups("MPI_Group_difference", group1, group2, newgroup, &a, &b);
    if (rc != MPI_SUCCESS) return fail("MPI_Group_difference", rc);
    std::set<int> in_b(b.begin(), b.end());
    std::vector<int> out;
    for (int x : a)
        if (!in_b.count(x)) out.push_back(x);
    return fail("MPI_Group_difference", group_create(out, newgroup));
}

// api/mpi_group.cpp:1288-1430: MPI_UNDEFINED for a process group2 lacks;
// MPI_PROC_NULL maps to itself (unless group2 is empty: the reference's
// translation loop never runs then, and every entry stays MPI_UNDEFINED)
MSX_EXPORT int MPI_Group_translate_ranks(MPI_Group group1, int n, const int ranks1[], MPI_Group group2,
                                         int ranks2[])
{
    api_require_init("MPI_Group_translate_ranks");
    std::vector<int> a, b;
    int rc = lookup(group1, &a);
    if (rc == MPI_SUCCESS) rc = lookup(group2, &b);
    if (rc == MPI_SUCCESS && n < 0) { set_error("**argneg n %d", n); rc = MPI_ERR_ARG; }
    if (rc != MPI_SUCCESS) return fail("MPI_Group_translate_ranks", rc);
    if (n == 0) return MPI_SUCCESS;
    if (!ranks1) { set_error("null ranks1"); return fail("MPI_Group_translate_ranks", MPI_ERR_ARG); }
    if (!ranks2) { set_error("null ranks2"); return fail("MPI_Group_translate_ranks", MPI_ERR_ARG); }
    for (int i = 0; i < n; ++i)
        if ((ranks1[i] < 0 && ranks1[i] != MPI_PROC_NULL) || (ranks1[i] >= 0 && (size_t)ranks1[i] >= a.size())) {
            set_error("**rank %d %zu", ranks1[i], a.size());
            return fail("MPI_Group_translate_ranks", MPI_ERR_RANK);
        }
    for (int i = 0; i < n; ++i) {
        ranks2[i] = MPI_UNDEFINED;
        if (b.empty()) continue;
        if (ranks1[i] == MPI_PROC_NULL) ranks2[i] = MPI_PROC_NULL;
        else ranks2[i] = rank_in(b, a[(size_t)ranks1[i]]);
    }
    return MPI_SUCCESS;
}

// api/mpi_group.cpp:35-135
MSX_EXPORT int MPI_Group_compare(MPI_Group group1, MPI_Group group2, int* result)
{
    api_require_init("MPI_Group_compare");
    std::vector<int> a, b;
    int rc = lookup(group1, &a);
    if (rc == MPI_SUCCESS) rc = lookup(group2, &b);
    if (rc == MPI_SUCCESS && !result) { set_error("null result"); rc = MPI_ERR_ARG; }
    if (rc != MPI_SUCCESS) return fail("MPI_Group_compare", rc);
    if (a.size() != b.size()) { *result = MPI_UNEQUAL; return MPI_SUCCESS; }
    std::vector<int> sa = a, sb = b;
    std::sort(sa.begin(), sa.end());
    std::sort(sb.begin(), sb.end());
    if (sa != sb) *result = MPI_UNEQUAL;
    else *result = a == b ? MPI_IDENT : MPI_SIMILAR;
    return MPI_SUCCESS;
}

#define MSX_ALIAS(name) extern "C" __attribute__((visibility("default"), alias(#name)))
MSX_ALIAS(MPI_Comm_group) int PMPI_Comm_group(MPI_Comm, MPI_Group*);
MSX_ALIAS(MPI_Group_size) int PMPI_Group_size(MPI_Group, int*);
MSX_ALIAS(MPI_Group_rank) int PMPI_Group_rank(MPI_Group, int*);
MSX_ALIAS(MPI_Group_free) int PMPI_Group_free(MPI_Group*);
MSX_ALIAS(MPI_Group_incl) int PMPI_Group_incl(MPI_Group, int, const int[], MPI_Group*);
MSX_ALIAS(MPI_Group_excl) int PMPI_Group_excl(MPI_Group, int, const int[], MPI_Group*);
MSX_ALIAS(MPI_Group_range_incl) int PMPI_Group_range_incl(MPI_Group, int, int[][3], MPI_Group*);
MSX_ALIAS(MPI_Group_range_excl) int PMPI_Group_range_excl(MPI_Group, int, int[][3], MPI_Group*);
MSX_ALIAS(MPI_Group_union) int PMPI_Group_union(MPI_Group, MPI_Group, MPI_Group*);
MSX_ALIAS(MPI_Group_intersection) int PMPI_Group_intersection(MPI_Group, MPI_Group, MPI_Group*);
MSX_ALIAS(MPI_Group_difference) int PMPI_Group_difference(MPI_Group, MPI_Group, MPI_Group*);
MSX_ALIAS(MPI_Group_translate_ranks) int PMPI_Group_translate_ranks(MPI_Group, int, const int[], MPI_Group, int[]);
MSX_ALIAS(MPI_Group_compare) int PMPI_Group_compare(MPI_Group, MPI_Group, int*);
