// sg_fast_att.hip — the Attention-pooling instantiations of the fused pair kernel
// (GCN → GCN → Attention(16) → NTN(16), layers.py:143-160 + 282-310).  The kernel
// template and host code are sg_fast.hip's; this translation unit compiles them with
// SG_FAST_ATT_TU so that only the Attention kernels are instantiated here and the
// default-stack ones there, and the two objects build in parallel.
#define SG_FAST_ATT_TU 1
#include "sg_fast.hip"
