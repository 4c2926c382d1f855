// msx_tree_bit.hip — k_tree launchers (BAND, BOR, BXOR), see msx_tree_impl.h.
// One translation unit per op family so the instantiations compile in parallel.
#include "msx_tree_impl.h"

namespace msx {

template hipError_t tree_dispatch<O_BAND>(Kind, const dev::TreeArgs&, int, void*, size_t, hipStream_t);
template hipError_t tree_dispatch<O_BOR>(Kind, const dev::TreeArgs&, int, void*, size_t, hipStream_t);
template hipError_t tree_dispatch<O_BXOR>(Kind, const dev::TreeArgs&, int, void*, size_t, hipStream_t);

}  // namespace msx
