// svao_fast.hip -- the SVAO "AO 1" / "AO 2" kernels of svao_kernels.h with fast numerics (rsd::fast,
// RSD_NUMERICS_FAST, the product default): compiled with FMA contraction, the hardware's approximate
// division / square root and float32 denormals flushed (Makefile FASTFLAGS).  D3D lets the reference's
// HLSL do exactly these (mad may fuse, '/' within 2.5 ulp, float32 denormals flush), so the result is
// graded against the CPU oracle by BASELINE.md section 4's AO tolerance instead of bit identity
// (tests/test_gpu_numerics.py).  The entry points and launch geometry stay in svao.hip.
#define RSD_FAST_NUMERICS 1
#include <hip/hip_runtime.h>

#include "rsd_device.h"
#include "rsd_internal.h"
#include "svao_math.h"

#define RSD_SVAO_NS fast
#include "svao_kernels.h"
