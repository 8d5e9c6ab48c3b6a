// jmme_tq_internal.h -- launchers of the transform / quant / SATD kernels
// (csrc/jmme_tq.hip); not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "jmme.h"

namespace jmme {

int transform_elems(int op);   // elements per block of op, 0 if unknown
hipError_t launch_transform(int op, const int32_t *in, int32_t *out, int n, hipStream_t s);
hipError_t launch_satd(int size, const int16_t *diff, int32_t *out, int n, hipStream_t s);
hipError_t launch_quant4x4(const jmme_quant4x4_params *params, const int32_t *param_idx, int32_t *coef, int32_t *levels,
                           int32_t *runs, int32_t *coeff_cost, int32_t *nonzero, int n, hipStream_t s);
hipError_t launch_residual4x4(const jmme_quant4x4_params *params, const jmme_resid4x4_req *req,
                              jmme_resid4x4_res *res, int n, hipStream_t s);

}  // namespace jmme
