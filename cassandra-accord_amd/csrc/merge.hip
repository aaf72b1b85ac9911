// merge.hip — batched KeyDeps.merge (placeholder until the union kernels land).
#include "prims.hpp"
namespace acc {
void keydeps_merge(acc_ctx *ctx, const acc_merge_in *in, acc_merge_view *view)
{
    (void)ctx; (void)in; (void)view;
    fail(ACC_E_STATE, "acc_keydeps_merge: not implemented in this build");
}
}  // namespace acc
