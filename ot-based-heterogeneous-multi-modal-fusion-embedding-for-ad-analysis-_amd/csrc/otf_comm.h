// otf_comm.h — internal interface of otf_comm.hip (RCCL resolved at run time).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "otfuse.h"

namespace otf {
// in-place all-reduce (OTF_RED_SUM / OTF_RED_MAX) of `count` elements of `dtype`
int comm_all_reduce(void* buf, int64_t count, int32_t dtype, int32_t op, otf_comm* comm,
                    hipStream_t s);
}  // namespace otf
