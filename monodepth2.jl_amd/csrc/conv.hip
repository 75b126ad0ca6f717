// Implicit-GEMM conv: weight packing, planning, workspace sizing, act_backward (see conv_impl.inc).
#define MD2_CONV_PART 0
#include "conv_impl.inc"
