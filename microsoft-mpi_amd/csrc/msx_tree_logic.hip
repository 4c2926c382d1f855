// msx_tree_logic.hip — k_tree launchers (logical and bitwise ops), see msx_tree_impl.h.
#include "msx_tree_impl.h"

namespace msx {

template hipError_t tree_dispatch<O_LAND>(Kind, const dev::TreeArgs&, int, void*, size_t, hipStream_t);
template hipError_t tree_dispatch<O_LOR>(Kind, const dev::TreeArgs&, int, void*, size_t, hipStream_t);
template hipError_t tree_dispatch<O_LXOR>(Kind, const dev::TreeArgs&, int, void*, size_t, hipStream_t);
template hipError_t tree_dispatch<O_BAND>(Kind, const dev::TreeArgs&, int, void*, size_t, hipStream_t);
template hipError_t tree_dispatch<O_BOR>(Kind, const dev::TreeArgs&, int, void*, size_t, hipStream_t);
template hipError_t tree_dispatch<O_BXOR>(Kind, const dev::TreeArgs&, int, void*, size_t, hipStream_t);

}  // namespace msx
