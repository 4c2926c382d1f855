// msx_tree_max.hip — k_tree launchers (MAX), see msx_tree_impl.h.
// One translation unit per op family so the instantiations compile in parallel.
#include "msx_tree_impl.h"

namespace msx {

template hipError_t tree_dispatch<O_MAX>(Kind, const dev::TreeArgs&, int, void*, size_t, hipStream_t);

}  // namespace msx
