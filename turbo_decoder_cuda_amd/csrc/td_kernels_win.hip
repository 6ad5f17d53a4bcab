// td_kernels_win.hip -- the sub-block (windowed) schedule of td_kernels.hip in a translation unit of
// its own, so that build.py can compile it with the max-ILP machine scheduler
// (-amdgpu-sched-strategy=max-ilp: the kernels issue each step's LDS table reads together; +1.4 % at
// BASELINE config 5) while the exact kernels keep the default scheduler (1 % slower
// under max-ILP).
#define TD_WIN_TU 1
#include "td_kernels.hip"
