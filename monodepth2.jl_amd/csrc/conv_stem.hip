// Implicit-GEMM conv: the ResNet stem forward on the space-to-depth grid (conv_stem.inc).
#define MD2_CONV_PART 5
#include "conv_impl.inc"
