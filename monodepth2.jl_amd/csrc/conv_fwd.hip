// Implicit-GEMM conv: forward pass launchers (see conv_impl.inc).
#define MD2_CONV_PART 1
#include "conv_impl.inc"
