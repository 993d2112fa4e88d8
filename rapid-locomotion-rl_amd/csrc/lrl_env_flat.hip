// lrl_env_flat.hip — the plane build of the env step kernel: lrl_env.hip with 4 envs per single-wave workgroup and
// 16 lanes (4 mirrored quads) per env (see the layout note at the top of lrl_env.hip).  Only env_step_kernel<false>
// and its entry points (lrl_launch_env_step_flat, lrl_env_kernel_setup_flat, lrl_debug_env_profile_flat) come from
// this translation unit; lrl_env.hip's lrl_launch_env_step dispatches the plane to it.
#define LRL_ENV_FLAT_TU
#include "lrl_env.hip"
