// msx_tree_cmp.hip — k_tree launchers (MAX, MIN, MAXLOC, MINLOC), see msx_tree_impl.h.
#include "msx_tree_impl.h"

namespace msx {

template hipError_t tree_dispatch<O_MAX>(Kind, const dev::TreeArgs&, int, void*, size_t, hipStream_t);
template hipError_t tree_dispatch<O_MIN>(Kind, const dev::TreeArgs&, int, void*, size_t, hipStream_t);
template hipError_t tree_dispatch<O_MAXLOC>(Kind, const dev::TreeArgs&, int, void*, size_t, hipStream_t);
template hipError_t tree_dispatch<O_MINLOC>(Kind, const dev::TreeArgs&, int, void*, size_t, hipStream_t);

}  // namespace msx
