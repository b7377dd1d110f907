// fp16 instance of the fused projection backward (k_pwl_bwd.hip), built without SLP vectorisation
// (Makefile: -fno-slp-vectorize for this file only; see the note at k_pwl_bwd.hip's instantiations)
#define DFD_PWL_F16_TU 1
#include "k_pwl_bwd.hip"
