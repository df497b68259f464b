// gs_sweep_ek4.hip — the EK = 4 (four-symbol DNA, no other symbols) instantiations of
// gs_sweep_kernel, compiled as their own translation unit beside gs_sweep.hip.
#define GS_SWEEP_EK4_UNIT
#include "gs_sweep.hip"
