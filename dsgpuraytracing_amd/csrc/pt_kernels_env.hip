// pt_kernels_env.hip -- the environment-light (ENV) instantiations of
// render_kernel (pt_kernels.hip), in their own translation unit so that they
// are compiled with the default instruction scheduler while the common build
// uses iterative-ILP scheduling (build.py).
#define PT_ENV_TU 1
#include "pt_kernels.hip"
