// Implicit-GEMM conv: filter-gradient pass launchers (see conv_impl.inc).
#define MD2_CONV_PART 3
#include "conv_impl.inc"
