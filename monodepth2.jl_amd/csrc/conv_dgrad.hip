// Implicit-GEMM conv: data-gradient pass launchers (see conv_impl.inc).
#define MD2_CONV_PART 2
#include "conv_impl.inc"
