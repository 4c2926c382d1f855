// msx_tree_sum.hip — k_tree launchers (SUM), see msx_tree_impl.h.
#include "msx_tree_impl.h"

namespace msx {

template hipError_t tree_dispatch<O_SUM>(Kind, const dev::TreeArgs&, int, void*, size_t, hipStream_t);

}  // namespace msx
