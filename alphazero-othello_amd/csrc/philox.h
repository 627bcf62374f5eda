// philox.h — counter-based RNG (Philox4x32-10) for the device-side draws of the self-play
// engine: Dirichlet root noise (MCTS_model.py:340-343), the temperature-0 tie break
// (:250-251), the action sample (self_play_worker.py:75), random D4 transforms and rollouts
// (:276-303).  Counter-based, so every game slot / rank has an independent, replayable
// stream without any per-thread state in HBM: counter = (slot, event, sub-draw, stream_id),
// key = seed.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bitboard.h"

namespace azr {

struct U4 {
  uint32_t x, y, z, w;
};

AZ_HD uint32_t mulhilo(uint32_t a, uint32_t b, uint32_t* hi) {
  const uint64_t p = (uint64_t)a * (uint64_t)b;
  *hi = (uint32_t)(p >> 32);
  return (uint32_t)p;
}

AZ_HD U4 philox(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, hi1;
    const uint32_t lo0 = mulhilo(0xD2511F53u, c.x, &hi0);
    const uint32_t lo1 = mulhilo(0xCD9E8D57u, c.z, &hi1);
    c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// Two independent doubles in [0, 1) with 53 random bits each.
AZ_HD void uniform2(uint64_t seed, uint32_t slot, uint32_t event, uint32_t sub, uint32_t stream,
                    double* a, double* b) {
  const U4 r = philox(U4{slot, event, sub, stream}, (uint32_t)seed, (uint32_t)(seed >> 32));
  const uint64_t x = ((uint64_t)r.x << 32) | r.y;
  const uint64_t y = ((uint64_t)r.z << 32) | r.w;
  *a = (double)(x >> 11) * (1.0 / 9007199254740992.0);
  *b = (double)(y >> 11) * (1.0 / 9007199254740992.0);
}

AZ_HD double uniform1(uint64_t seed, uint32_t slot, uint32_t event, uint32_t sub,
                      uint32_t stream) {
  double a, b;
  uniform2(seed, slot, event, sub, stream, &a, &b);
  return a;
}

// Gamma(alpha, 1) by Marsaglia-Tsang (alpha < 1 via the alpha+1 boost).  Each call
// consumes sub-draws sub*64 + i of its own counter range, so lanes never share draws.
__device__ inline double gamma_draw(double alpha, uint64_t seed, uint32_t slot, uint32_t event,
                                    uint32_t sub, uint32_t stream) {
  const bool boost = alpha < 1.0;
  const double a = boost ? alpha + 1.0 : alpha;
  const double d = a - 1.0 / 3.0;
  const double c = 1.0 / sqrt(9.0 * d);
  double g = 0.0;
  for (uint32_t i = 0; i < 64; ++i) {
    double u1, u2;
    uniform2(seed, slot, event, sub * 64u + i, stream, &u1, &u2);
    // Box-Muller normal from (u1, u2); u1 in (0, 1]
    const double x = sqrt(-2.0 * log(1.0 - u1)) * cospi(2.0 * u2);
    double v = 1.0 + c * x;
    if (v <= 0.0) continue;
    v = v * v * v;
    double u3, u4;
    uniform2(seed, slot, event, sub * 64u + i, stream ^ 0x80000000u, &u3, &u4);
    if (log(1.0 - u3) < 0.5 * x * x + d - d * v + d * log(v)) {
      g = d * v;
      if (boost) g *= pow(1.0 - u4, 1.0 / alpha);
      return g;
    }
  }
  return d;  // practically unreachable (acceptance rate > 95% per trial)
}

}  // namespace azr
