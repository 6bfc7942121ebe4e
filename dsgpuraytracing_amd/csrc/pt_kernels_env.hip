// pt_kernels_env.hip -- the environment-light (ENV) instantiations of
// render_kernel (pt_kernels.hip), in their own translation unit so that each
// build gets its own machine scheduler: iterative-ILP here, max-ILP for the
// common build (build.py: PT_ENV_SCHED / PT_KERNEL_SCHED).
#define PT_ENV_TU 1
#include "pt_kernels.hip"
