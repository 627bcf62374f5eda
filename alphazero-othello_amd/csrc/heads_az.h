// heads_az.h — AlphaZeroNet's policy and value heads for NB = 4 (or 2) boards of a
// workgroup's four waves, one wavefront per board for the 1x1 convs, shared by the stand-alone heads kernel (heads.hip, trunk output read from global
// memory) and the last trunk conv with the heads fused into its epilogue (conv_wino4.hip,
// trunk output read from LDS).  Both feed the same registers to the same code, so the two
// paths give bit-identical priors and values.
//
// Reference Models.py:164-221 (inference copy, BatchNorm folded into the 1x1 convs):
//   p = relu(conv1x1_{C->2}(h) + b)            flattened NCHW: p[c*64 + pos]
//   logits = pol_fc(p)  (128 -> 65)            priors = softmax(logits)  (MCTS_model.py:319)
//   v = relu(conv1x1_{C->1}(h) + b)            v[pos]
//   value = tanh(val_fc2(relu(val_fc1(v))))   (64 -> 256 -> 1)
// Lane = board square for the 1x1 convs.  The FCs are split by INPUT range over the four
// waves, each computing its quarter for all NB boards (pol_fc^T [128][65]: inputs
// 32w..32w+31; val_fc1^T [64][256]: inputs 16w..16w+15), so every FC weight is read from L2
// once per NB boards; the partial sums meet in LDS and wave b adds them in order for
// board b.  The quarters and their order do not depend on NB, so every NB gives the same
// bits (the two-board form is the fused epilogue of the two-board trunk conv).
#pragma once
#include <hip/hip_runtime.h>

#ifndef AZ_HEADS_CHECK
#define AZ_HEADS_CHECK 0
#endif


namespace azh {

constexpr int kBoards = 4;  // boards per workgroup of the stand-alone kernel
constexpr int kQuarters = 4;  // waves splitting the FC inputs (any NB <= 4 boards)

struct Weights {
  const float* wpv;    // [3][C]: policy ch 0, policy ch 1, value
  const float* bpv;    // [3]
  const float* wpolT;  // [128][65]
  const float* bpol;   // [65]
  const float* w1T;    // [64][256]
  const float* b1;     // [256]
  const float* w2;     // [256]
  const float* b2;     // [1]
};

// LDS the four waves exchange partial sums through (NB = 4: 3 KiB + 20.3 KiB); `p` / `v`
// are written while other waves may still be reading their activations, the rest only
// after the first barrier
template <int NB = kBoards>
struct ScratchT {
  float (*p)[128];             // [NB][128] relu'd policy 1x1 conv, NCHW-flat
  float (*v)[64];              // [NB][64] relu'd value 1x1 conv
  float (*lp)[NB][65];         // [quarter][board][logit] partial logits
  float4 (*hv)[NB][64];        // [quarter][board][lane] partial val_fc1 hidden units
};
using Scratch = ScratchT<kBoards>;

// The four components of a float4 accumulator kept as four separate fp32 chains.  Left to
// itself the compiler pairs them into v_pk_mul_f32 / v_pk_add_f32 (SLP); in the val_fc1
// partial sums below those packed chains gave wrong words -- in lanes 48-63 only, in a few
// boards per launch, and only with two two-board workgroups resident on a CU (round 3's
// "values, never priors" on the two-board heads).  Located in round 4 with the AZ_HEADS_CHECK
// build (every wave recomputes its value path from its own registers and names each
// differing word: only lanes 48-63 of the partial-sum quads, profiles/r04_heads_war.json);
// an A/B of fixes (profiles/r04_heads_fix_ab.json): waiting for the FC weights before use
// leaves the errors, unpaired chains (this) remove them in every heads test and stress run.
// An empty asm with the four values as read-write operands stops the pairing; the float
// operations and their order are unchanged.
#ifndef AZ_HEADS_UNPAIRED
#define AZ_HEADS_UNPAIRED 1  // 0: round 3's code (the failing form, for the ISA analysis)
#endif
__device__ __forceinline__ void unpaired(float4& a) {
  if constexpr (AZ_HEADS_UNPAIRED) asm volatile("" : "+v"(a.x), "+v"(a.y), "+v"(a.z), "+v"(a.w));
}

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}
__device__ __forceinline__ float wave_max(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = fmaxf(x, __shfl_xor(x, o, 64));
  return x;
}

// Wave w < 4 of the workgroup computes FC quarter w (any further waves of a larger
// workgroup pass active = false and only take part in the two barriers); waves w < NB also
// own board w: xf(c) = channels 4c..4c+3 of board w's activations at square `lane`
// (registers loaded up front, or LDS read on demand), b = that board's index, live = it
// exists (false for w >= NB).
template <int C, int NB = kBoards, class XF>
__device__ __forceinline__ void heads_four(XF&& xf, int lane, int w, int b, bool live,
                                           bool active, const Weights& W,
                                           const ScratchT<NB>& L, float* __restrict__ priors,
                                           float* __restrict__ values) {
  static_assert(NB >= 1 && NB <= kQuarters, "boards per workgroup");
  constexpr int KP = 128 / kQuarters, KV = 64 / kQuarters;  // FC inputs per wave
  float wpl[KP];
  float w64 = 0.f;
  float4 wq[KV];
  if (active) {
#pragma unroll
    for (int k = 0; k < KP; ++k) wpl[k] = W.wpolT[(KP * w + k) * 65 + lane];
    w64 = lane < KP ? W.wpolT[(KP * w + lane) * 65 + 64] : 0.f;
#pragma unroll
    for (int i = 0; i < KV; ++i)
      wq[i] = reinterpret_cast<const float4*>(W.w1T + (KV * w + i) * 256)[lane];
  }
#if AZ_HEADS_CHECK
  float myv = 0.f;  // debug builds: this wave's own value 1x1 output, kept in a register
#endif
  if (active && w < NB) {
    // 1x1 convs (policy 2 channels, value 1 channel) of board w at square `lane`
    float d0 = 0.f, d1 = 0.f, d2 = 0.f;
    const float4* w0 = reinterpret_cast<const float4*>(W.wpv);
    const float4* w1 = reinterpret_cast<const float4*>(W.wpv + C);
    const float4* w2v = reinterpret_cast<const float4*>(W.wpv + 2 * C);
#pragma unroll
    for (int c = 0; c < C / 4; ++c) {
      const float4 a = w0[c], q = w1[c], r = w2v[c], xc = xf(c);
      d0 += xc.x * a.x + xc.y * a.y + xc.z * a.z + xc.w * a.w;
      d1 += xc.x * q.x + xc.y * q.y + xc.z * q.z + xc.w * q.w;
      d2 += xc.x * r.x + xc.y * r.y + xc.z * r.z + xc.w * r.w;
    }
    L.p[w][lane] = fmaxf(d0 + W.bpv[0], 0.f);
    L.p[w][64 + lane] = fmaxf(d1 + W.bpv[1], 0.f);
    L.v[w][lane] = fmaxf(d2 + W.bpv[2], 0.f);
#if AZ_HEADS_CHECK
    myv = fmaxf(d2 + W.bpv[2], 0.f);
#endif
  }
  __syncthreads();

  // this wave's input quarter of both FCs, for every board of the workgroup
  if (active) {
#pragma unroll
    for (int bd = 0; bd < NB; ++bd) {
      float la = 0.f;
#pragma unroll
      for (int k = 0; k < KP; ++k) la += wpl[k] * L.p[bd][KP * w + k];
      L.lp[w][bd][lane] = la;
      const float l64 = wave_sum(lane < KP ? w64 * L.p[bd][KP * w + lane] : 0.f);
      if (lane == 0) L.lp[w][bd][64] = l64;
      float4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < KV; ++i) {
        const float vi = L.v[bd][KV * w + i];
        acc.x += wq[i].x * vi;
        acc.y += wq[i].y * vi;
        acc.z += wq[i].z * vi;
        acc.w += wq[i].w * vi;
        unpaired(acc);
      }
      L.hv[w][bd][lane] = acc;
#if AZ_HEADS_CHECK
      {  // debug builds: the quad recomputed from fresh weight loads, and read back
        float4 acc2 = {0.f, 0.f, 0.f, 0.f};
        for (int i = 0; i < KV; ++i) {
          const float vi = L.v[bd][KV * w + i];
          const float4 wi = reinterpret_cast<const float4*>(W.w1T + (KV * w + i) * 256)[lane];
          acc2.x += wi.x * vi;
          acc2.y += wi.y * vi;
          acc2.z += wi.z * vi;
          acc2.w += wi.w * vi;
          if (wi.x != wq[i].x || wi.y != wq[i].y || wi.z != wq[i].z || wi.w != wq[i].w)
            printf("HEADS_CHECK wq wg %d wave %d q %d i %d lane %d reg %a fresh %a\n",
                   (int)blockIdx.x, (int)(threadIdx.x >> 6), w, i, lane, wq[i].x, wi.x);
        }
        if (acc2.x != acc.x || acc2.y != acc.y || acc2.z != acc.z || acc2.w != acc.w)
          printf("HEADS_CHECK acc wg %d wave %d q %d bd %d lane %d reg %a fresh %a\n",
                 (int)blockIdx.x, (int)(threadIdx.x >> 6), w, bd, lane, acc.x, acc2.x);
        const float4 rb = L.hv[w][bd][lane];
        if (rb.x != acc.x || rb.y != acc.y || rb.z != acc.z || rb.w != acc.w)
          printf("HEADS_CHECK store wg %d wave %d q %d bd %d lane %d lds %a reg %a\n",
                 (int)blockIdx.x, (int)(threadIdx.x >> 6), w, bd, lane, rb.x, acc.x);
      }
#endif
    }
  }
  __syncthreads();
  if (!active || !live || w >= NB) return;  // whole wave (uniform); no barrier follows

  // board w: the quarters added in order, softmax over the 65 logits
  float la = W.bpol[lane], l64 = W.bpol[64];
#pragma unroll
  for (int q = 0; q < kQuarters; ++q) {
    la += L.lp[q][w][lane];
    l64 += L.lp[q][w][64];
  }
  const float m = fmaxf(wave_max(la), l64);
  const float e = __expf(la - m), e64 = __expf(l64 - m);
  const float inv = 1.f / (wave_sum(e) + e64);
  priors[(size_t)b * 65 + lane] = e * inv;
  if (lane == 0) priors[(size_t)b * 65 + 64] = e64 * inv;

  // value: lane j -> hidden units 4j..4j+3 of val_fc1, then val_fc2 reduced over the wave
  float4 acc = reinterpret_cast<const float4*>(W.b1)[lane];
#pragma unroll
  for (int q = 0; q < kQuarters; ++q) {
    const float4 a = L.hv[q][w][lane];
    acc.x += a.x;
    acc.y += a.y;
    acc.z += a.z;
    acc.w += a.w;
    unpaired(acc);
  }
  const float4 o = reinterpret_cast<const float4*>(W.w2)[lane];
  const float part = fmaxf(acc.x, 0.f) * o.x + fmaxf(acc.y, 0.f) * o.y +
                     fmaxf(acc.z, 0.f) * o.z + fmaxf(acc.w, 0.f) * o.w;
  const float val = wave_sum(part) + W.b2[0];
  if (lane == 0) values[b] = tanhf(val);
#if AZ_HEADS_CHECK
  // debug builds: the value path recomputed by this wave alone from its own registers (no
  // LDS), in the same order; every differing word named
  if (L.v[w][lane] != myv)
    printf("HEADS_CHECK v wg %d wave %d board %d lane %d lds %a reg %a\n", (int)blockIdx.x,
           (int)(threadIdx.x >> 6), b, lane, L.v[w][lane], myv);
  float4 chk = reinterpret_cast<const float4*>(W.b1)[lane];
  for (int q = 0; q < kQuarters; ++q) {
    float4 pq = {0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < KV; ++i) {
      const float vi = __shfl(myv, KV * q + i, 64);
      const float4 wi = reinterpret_cast<const float4*>(W.w1T + (KV * q + i) * 256)[lane];
      pq.x += wi.x * vi;
      pq.y += wi.y * vi;
      pq.z += wi.z * vi;
      pq.w += wi.w * vi;
    }
    const float4 a = L.hv[q][w][lane];
    if (a.x != pq.x || a.y != pq.y || a.z != pq.z || a.w != pq.w)
      printf("HEADS_CHECK hv wg %d wave %d board %d q %d lane %d lds %a %a reg %a %a\n",
             (int)blockIdx.x, (int)(threadIdx.x >> 6), b, q, lane, a.x, a.y, pq.x, pq.y);
    chk.x += pq.x;
    chk.y += pq.y;
    chk.z += pq.z;
    chk.w += pq.w;
  }
  const float part2 = fmaxf(chk.x, 0.f) * o.x + fmaxf(chk.y, 0.f) * o.y +
                      fmaxf(chk.z, 0.f) * o.z + fmaxf(chk.w, 0.f) * o.w;
  const float val2 = wave_sum(part2) + W.b2[0];
  if (lane == 0 && val2 != val)
    printf("HEADS_CHECK val wg %d wave %d board %d lds %a reg %a\n", (int)blockIdx.x,
           (int)(threadIdx.x >> 6), b, val, val2);
#endif
}

}  // namespace azh
