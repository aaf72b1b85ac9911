// levelise.hip — executeAt levelisation (placeholder until the wavefront kernels land).
#include "prims.hpp"
namespace acc {
void levelise(acc_ctx *ctx, const acc_graph_in *in, uint32_t *level, uint32_t *order, uint32_t *n_levels)
{
    (void)ctx; (void)in; (void)level; (void)order; (void)n_levels;
    fail(ACC_E_STATE, "acc_levelise: not implemented in this build");
}
}  // namespace acc
