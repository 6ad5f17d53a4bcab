// td_kernels_w12.hip -- td_kernels.hip again with 12-step windows, in namespace td_w12, for the fp32
// turbo kernel at four workgroups per CU (td::launch_turbo4_w12): with the default 15-step windows the
// fp32 workgroup's LDS fits three per CU, with 12 it fits four (large batches).
#define TD_W12_TU 1
#define TD_KW 12
#include "td_kernels.hip"
