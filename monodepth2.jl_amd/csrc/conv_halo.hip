// Implicit-GEMM conv: the LDS-halo stride-1 3x3 fwd / dgrad kernel (conv_halo.inc).
#define MD2_CONV_PART 4
#include "conv_impl.inc"
