// The --math exact instantiations of the deep sweep (k_tbn, hip_tbn.hip) in an object of their
// own: built under LLVM's max-memory-clause machine scheduler, which runs the exact sweep ~1.3 %
// faster than max-ilp, while the fma sweep (the headline) keeps max-ilp (profiles/deep_sweeps_r5.txt
// step 14). hip_tbn.hip's launcher takes these kernels through tbn_exact_kernel().
#define W3D_TBN_PART 2
#include "hip_tbn.hip"
