// bs_prelude.hpp -- gfx950 primitives for the generated bitsliced AES round
// (bs_aes.hpp, tools/gen_bitslice.py) and the bitsliced Meow chain
// (bs_meow.hpp).  The same two headers compile for the host test harness
// (tests/cpp/bs_host_test.cpp) against that harness's own prelude.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define KVH_BS_DEV __device__ __forceinline__

namespace kvh {
namespace bs {
// v_bitop3_b32: any 3-input boolean function, truth-table index a*4 + b*2 + c
template <uint32_t TT>
KVH_BS_DEV uint32_t bop3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, TT);
}
// v_alignbit_b32: ({hi, lo} >> s)[31:0]
KVH_BS_DEV uint32_t alignbit(uint32_t hi, uint32_t lo, uint32_t s) { return __builtin_amdgcn_alignbit(hi, lo, s); }
// v_perm_b32: byte k of the result = byte sel_k of {hi, lo} (0-3 lo, 4-7 hi)
KVH_BS_DEV uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) { return __builtin_amdgcn_perm(hi, lo, sel); }
// wave-uniform value of lane t of a VGPR (v_readlane_b32 -> SGPR)
KVH_BS_DEV uint32_t lane_val(uint32_t v, uint32_t t) { return __builtin_amdgcn_readlane(v, t); }
}  // namespace bs
}  // namespace kvh

#include "bs_aes.hpp"
#include "bs_meow.hpp"
