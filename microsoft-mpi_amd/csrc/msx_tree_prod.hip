// msx_tree_prod.hip — k_tree launchers (PROD), see msx_tree_impl.h.
// One translation unit per op family so the instantiations compile in parallel.
#include "msx_tree_impl.h"

namespace msx {

template hipError_t tree_dispatch<O_PROD>(Kind, const dev::TreeArgs&, int, void*, size_t, hipStream_t);

}  // namespace msx
