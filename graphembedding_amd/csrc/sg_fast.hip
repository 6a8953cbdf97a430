// sg_fast.hip — placeholder until the fused kernel lands.
#include "sg_plan.h"
int sg_fast_supported(const sg_model_t *, const SgGenPlan &) { return 0; }
int64_t sg_fast_slab_floats(const SgGenPlan &, int64_t) { return 0; }
int sg_fast_run(const sg_model_t *, const SgGenPlan &, bool, const void *, int64_t, int64_t,
                int64_t, const float *, uint64_t, const float *, float *, float *, int *,
                hipStream_t) { return SG_ERR_UNSUPPORTED; }
