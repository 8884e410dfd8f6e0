// Fused decode-step kernels around the decode GEMM (one launch each, replacing
// 5-20 framework kernels per op):
//   k_rmsnorm       y = bf16(bf16(x * rsqrt(mean(x^2) + eps)) * w)   one workgroup per row,
//                   optionally after a deferred GEMM's residual epilogue
//   k_rope_kv       q/k rotate-half RoPE at one position, k/v appended into the
//                   KV cache (and a second copy, the packed cache's raw tail)
//   k_attn_decode   GQA decode attention, flash-decoding split over the
//                   context: one workgroup per (batch, kv head, 256-token split)
//                   computes the group's 8 query heads' scores (lane = token),
//                   softmax partials and P.V (lane = head-dim pair) in f32;
//   k_attn_combine  merges the splits (log-sum-exp) and writes bf16.
// The KV cache layout is [2][B][Hkv][T][hd] (k then v), bf16.
#include <cstdlib>
#include <hip/hip_runtime.h>

#include "ogkm/kernels.hpp"

namespace ogkm {

__device__ __forceinline__ float dbf(uint16_t b) { return __uint_as_float((uint32_t)b << 16); }
__device__ __forceinline__ uint16_t df2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x7FFFFFu)) return (uint16_t)((u >> 16) | 0x40u);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---------------------------------------------------------------- RMSNorm (+ deferred residual GEMM epilogue)
// One 256-thread workgroup per row; thread t owns columns 4t + 1024 j of its G
// column groups (16-byte f32x4 partial loads, 8-byte bf16 loads/stores). With
// a.part set, the row first takes the deferred decode GEMM's RESID epilogue:
// x = bf16(bf16(sum_k part[k]) + x), summed k ascending like k_dgemm_reduce, so
// the fused and the separate path give identical bits - and one launch (this
// one) replaces the reduce + the norm. Every load is unconditional (clamped
// index, predicated use) and a batch of them is issued before the first use:
// a per-element load-or-zero select makes the compiler wait vmcnt(0) per
// element (one dependent round trip each). (A multi-workgroup form - one
// workgroup per 1024 columns, the row's last arriver normalising - measured
// slower: 11.2 vs 9.5 us, the release/acquire hand-off costs more than it
// spreads.)
__device__ __forceinline__ void norm_store4(const ResidNormArgs& a, uint32_t row, uint32_t c, const float (&x4)[4],
                                            uint2 wp, float r) {
  const float w4[4] = {dbf((uint16_t)wp.x), dbf((uint16_t)(wp.x >> 16)), dbf((uint16_t)wp.y),
                       dbf((uint16_t)(wp.y >> 16))};
  uint16_t o[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) o[e] = df2bf(dbf(df2bf(x4[e] * r)) * w4[e]);
  uint16_t* dst = a.y_frag ? a.y + frag_index(row, c, a.dim) : a.y + (uint64_t)row * a.ldy + c;
  *reinterpret_cast<uint2*>(dst) =
      uint2{(uint32_t)o[0] | ((uint32_t)o[1] << 16), (uint32_t)o[2] | ((uint32_t)o[3] << 16)};
}

// NT threads per row: 256 (G column groups of kNormCols), or 1024 for few-row
// (decode-batch) norms - four times the loads in flight per row, so the split-K
// partials of a 64-row residual take fewer dependent rounds (OGKM_NORM_1K=0:
// the 256-thread form only).
template <int G, int NT = 256>
__global__ void __launch_bounds__(NT) k_rmsnorm(ResidNormArgs a) {
  constexpr uint32_t kCols = 4 * NT;
  __shared__ float red[NT / 64];
  const uint32_t row = blockIdx.x, t = threadIdx.x;
  uint16_t* xr = a.x + (uint64_t)row * a.ldx;
  uint32_t cl[G];  // clamped column of each group (loads); c < dim gates the use
  bool on[G];
  uint2 xp[G], wp[G];
#pragma unroll
  for (int j = 0; j < G; ++j) {
    const uint32_t c = 4 * t + kCols * j;
    on[j] = c < a.dim;
    cl[j] = on[j] ? c : a.dim - 4;
    xp[j] = *reinterpret_cast<const uint2*>(xr + cl[j]);
    wp[j] = *reinterpret_cast<const uint2*>(a.w + cl[j]);
  }
  float v[G][4];
#pragma unroll
  for (int j = 0; j < G; ++j) {
    v[j][0] = dbf((uint16_t)xp[j].x);
    v[j][1] = dbf((uint16_t)(xp[j].x >> 16));
    v[j][2] = dbf((uint16_t)xp[j].y);
    v[j][3] = dbf((uint16_t)(xp[j].y >> 16));
  }
  if (a.part) {
    constexpr uint32_t KB = G <= 2 ? 16 : G <= 4 ? 8 : G <= 8 ? 4 : 2;  // splits per batch: KB x G loads in flight
    float4 sum[G];
#pragma unroll
    for (int j = 0; j < G; ++j) sum[j] = float4{0.f, 0.f, 0.f, 0.f};
    for (uint32_t k0 = 0; k0 < a.ksplit; k0 += KB) {
      float4 pv[KB][G];
#pragma unroll
      for (uint32_t kk = 0; kk < KB; ++kk) {
        const uint32_t k = k0 + kk < a.ksplit ? k0 + kk : a.ksplit - 1;
#pragma unroll
        for (int j = 0; j < G; ++j)
          pv[kk][j] = *reinterpret_cast<const float4*>(a.part + ((uint64_t)k * a.rows + row) * a.dim + cl[j]);
      }
#pragma unroll
      for (uint32_t kk = 0; kk < KB; ++kk) {
        const bool in = k0 + kk < a.ksplit;
#pragma unroll
        for (int j = 0; j < G; ++j) {
          sum[j].x = in ? sum[j].x + pv[kk][j].x : sum[j].x;
          sum[j].y = in ? sum[j].y + pv[kk][j].y : sum[j].y;
          sum[j].z = in ? sum[j].z + pv[kk][j].z : sum[j].z;
          sum[j].w = in ? sum[j].w + pv[kk][j].w : sum[j].w;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const float s4[4] = {sum[j].x, sum[j].y, sum[j].z, sum[j].w};
      uint16_t o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[e] = df2bf(dbf(df2bf(s4[e])) + v[j][e]);
        v[j][e] = dbf(o[e]);
      }
      if (on[j])
        *reinterpret_cast<uint2*>(xr + cl[j]) =
            uint2{(uint32_t)o[0] | ((uint32_t)o[1] << 16), (uint32_t)o[2] | ((uint32_t)o[3] << 16)};
    }
  }
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < G; ++j)
    ss = on[j] ? ss + v[j][0] * v[j][0] + v[j][1] * v[j][1] + v[j][2] * v[j][2] + v[j][3] * v[j][3] : ss;
  ss = wave_sum(ss);
  if ((t & 63) == 0) red[t >> 6] = ss;
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) tot += red[w];
  const float r = rsqrtf(tot / (float)a.dim + a.eps);
#pragma unroll
  for (int j = 0; j < G; ++j)
    if (on[j]) norm_store4(a, row, cl[j], v[j], wp[j], r);
}

// Two-launch RMSNorm for few rows (decode batches): a row's 1024-column blocks
// are spread over workgroups, so a 64-row norm runs on dim / 4 x 64 / 256
// workgroups instead of 64 (one per CU - latency-bound at ~8 us for the
// residual's split-K partials). k_norm_ssq: residual epilogue (as k_rmsnorm:
// x = bf16(bf16(sum_k part[k]) + x), k ascending) and the block's sum of
// squares into ssq[row][block]; k_norm_scale: r = rsqrt(sum of the row's block
// sums / dim + eps), y = bf16(bf16(x r) w). Deterministic (fixed summation
// order, no atomics).
__global__ void __launch_bounds__(256) k_norm_ssq(ResidNormArgs a) {
  __shared__ float red[4];
  const uint32_t row = blockIdx.y, t = threadIdx.x;
  const uint32_t c = blockIdx.x * kNormCols + 4 * t;
  const bool on = c < a.dim;
  const uint32_t cl = on ? c : a.dim - 4;
  uint16_t* xr = a.x + (uint64_t)row * a.ldx;
  const uint2 xp = *reinterpret_cast<const uint2*>(xr + cl);
  float v[4] = {dbf((uint16_t)xp.x), dbf((uint16_t)(xp.x >> 16)), dbf((uint16_t)xp.y), dbf((uint16_t)(xp.y >> 16))};
  if (a.part) {
    constexpr uint32_t KB = 16;  // splits in flight per batch
    float4 sum = float4{0.f, 0.f, 0.f, 0.f};
    for (uint32_t k0 = 0; k0 < a.ksplit; k0 += KB) {
      float4 pv[KB];
#pragma unroll
      for (uint32_t kk = 0; kk < KB; ++kk) {
        const uint32_t k = k0 + kk < a.ksplit ? k0 + kk : a.ksplit - 1;
        pv[kk] = *reinterpret_cast<const float4*>(a.part + ((uint64_t)k * a.rows + row) * a.dim + cl);
      }
#pragma unroll
      for (uint32_t kk = 0; kk < KB; ++kk) {
        const bool in = k0 + kk < a.ksplit;
        sum.x = in ? sum.x + pv[kk].x : sum.x;
        sum.y = in ? sum.y + pv[kk].y : sum.y;
        sum.z = in ? sum.z + pv[kk].z : sum.z;
        sum.w = in ? sum.w + pv[kk].w : sum.w;
      }
    }
    const float s4[4] = {sum.x, sum.y, sum.z, sum.w};
    uint16_t o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      o[e] = df2bf(dbf(df2bf(s4[e])) + v[e]);
      v[e] = dbf(o[e]);
    }
    if (on)
      *reinterpret_cast<uint2*>(xr + cl) =
          uint2{(uint32_t)o[0] | ((uint32_t)o[1] << 16), (uint32_t)o[2] | ((uint32_t)o[3] << 16)};
  }
  float ss = on ? v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3] : 0.f;
  ss = wave_sum(ss);
  if ((t & 63) == 0) red[t >> 6] = ss;
  __syncthreads();
  if (t == 0) a.ssq[(uint64_t)row * gridDim.x + blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void __launch_bounds__(256) k_norm_scale(ResidNormArgs a) {
  const uint32_t row = blockIdx.y, t = threadIdx.x;
  const uint32_t c = blockIdx.x * kNormCols + 4 * t;
  if (c >= a.dim) return;
  const uint32_t nb = gridDim.x;
  float tot = 0.f;
  for (uint32_t j = 0; j < nb; ++j) tot += a.ssq[(uint64_t)row * nb + j];
  const float r = rsqrtf(tot / (float)a.dim + a.eps);
  const uint2 xp = *reinterpret_cast<const uint2*>(a.x + (uint64_t)row * a.ldx + c);
  const uint2 wp = *reinterpret_cast<const uint2*>(a.w + c);
  const float v[4] = {dbf((uint16_t)xp.x), dbf((uint16_t)(xp.x >> 16)), dbf((uint16_t)xp.y),
                      dbf((uint16_t)(xp.y >> 16))};
  norm_store4(a, row, c, v, wp, r);
}

// ---------------------------------------------------------------- RoPE + KV append
// One thread per (b, head, i < hd/2) over the q heads, then the k heads (rotated,
// appended) and the v heads (appended).
__global__ void __launch_bounds__(256) k_rope_kv(RopeKvArgs a) {
  const uint32_t half = a.hd / 2;
  const uint32_t heads = a.hq + 2 * a.hkv;
  const uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (uint64_t)a.B * heads * half) return;
  const uint32_t i = (uint32_t)(idx % half);
  const uint32_t hh = (uint32_t)((idx / half) % heads);
  const uint32_t b = (uint32_t)(idx / ((uint64_t)half * heads));
  float x1, x2;
  if (a.part) {  // deferred qkv GEMM: its split-K sum + store epilogue, here
    const uint32_t n = heads * a.hd, c1 = hh * a.hd + i;
    float s1 = 0.f, s2 = 0.f;
    constexpr uint32_t kB = 8;  // splits in flight per batch (summed k ascending)
    for (uint32_t k0 = 0; k0 < a.ksplit; k0 += kB) {
      float p1[kB], p2[kB];
#pragma unroll
      for (uint32_t kk = 0; kk < kB; ++kk) {  // unconditional (clamped) loads, predicated adds
        const uint32_t k = k0 + kk < a.ksplit ? k0 + kk : a.ksplit - 1;
        const float* row = a.part + ((uint64_t)k * a.B + b) * n;
        p1[kk] = row[c1];
        p2[kk] = row[c1 + half];
      }
#pragma unroll
      for (uint32_t kk = 0; kk < kB; ++kk) {
        const bool in = k0 + kk < a.ksplit;
        s1 = in ? s1 + p1[kk] : s1;
        s2 = in ? s2 + p2[kk] : s2;
      }
    }
    x1 = dbf(df2bf(s1));
    x2 = dbf(df2bf(s2));
  } else {
    const uint16_t* src = a.qkv + (uint64_t)b * a.ldqkv + (uint64_t)hh * a.hd;
    x1 = dbf(src[i]);
    x2 = dbf(src[i + half]);
  }
  if (hh < a.hq + a.hkv) {
    const float c = a.cos[i], s = a.sin[i];
    const float r1 = x1 * c - x2 * s, r2 = x2 * c + x1 * s;
    x1 = r1;
    x2 = r2;
  }
  const uint16_t o1 = df2bf(x1), o2 = df2bf(x2);
  if (hh < a.hq) {
    uint16_t* q = a.q_out + ((uint64_t)b * a.hq + hh) * a.hd;
    q[i] = o1;
    q[i + half] = o2;
    return;
  }
  const uint32_t kv = hh < a.hq + a.hkv ? 0u : 1u;
  const uint32_t h = hh - a.hq - kv * a.hkv;
  uint16_t* c = a.cache + ((((uint64_t)kv * a.B + b) * a.hkv + h) * a.T + a.pos) * a.hd;
  c[i] = o1;
  c[i + half] = o2;
  if (a.tail) {
    uint16_t* t = a.tail + ((((uint64_t)kv * a.B + b) * a.hkv + h) * a.tail_T + a.tail_pos) * a.hd;
    t[i] = o1;
    t[i + half] = o2;
  }
}

// ---------------------------------------------------------------- attention
constexpr int kAttnSplit = 256;  // tokens per workgroup
constexpr int kMaxGroup = 16;    // query heads per kv head
constexpr int kMaxHd = 128;

__global__ void __launch_bounds__(256) k_attn_decode(AttnArgs a) {
  __shared__ float qs[kMaxGroup][kMaxHd];       // this kv head's query group, f32
  __shared__ float ps[kMaxGroup][kAttnSplit];   // scores -> probabilities
  __shared__ float ms[kMaxGroup], ls[kMaxGroup];
  __shared__ float part[4][kMaxGroup][kMaxHd / 2 * 2];  // per-wave P.V partials
  const uint32_t split = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const uint32_t g = a.hq / a.hkv;
  const uint32_t t0 = split * kAttnSplit;
  const uint32_t nt = a.len - t0 < (uint32_t)kAttnSplit ? a.len - t0 : (uint32_t)kAttnSplit;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (uint32_t e = tid; e < g * a.hd; e += 256) {
    const uint32_t h = e / a.hd, d = e - h * a.hd;
    qs[h][d] = dbf(a.q[((uint64_t)b * a.hq + kvh * g + h) * a.hd + d]) * a.scale;
  }
  __syncthreads();
  const uint16_t* kbase = a.cache + (((uint64_t)0 * a.B + b) * a.hkv + kvh) * (uint64_t)a.T * a.hd;
  const uint16_t* vbase = a.cache + (((uint64_t)1 * a.B + b) * a.hkv + kvh) * (uint64_t)a.T * a.hd;
  // scores: lane = token
  if (tid < nt) {
    const uint16_t* kr = kbase + (uint64_t)(t0 + tid) * a.hd;
    float acc[kMaxGroup];
#pragma unroll
    for (int h = 0; h < kMaxGroup; ++h) acc[h] = 0.f;
    for (uint32_t d = 0; d < a.hd; d += 8) {
      const uint4 kv8 = *reinterpret_cast<const uint4*>(kr + d);
      const uint32_t w4[4] = {kv8.x, kv8.y, kv8.z, kv8.w};
      float kf[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        kf[2 * j] = dbf((uint16_t)w4[j]);
        kf[2 * j + 1] = dbf((uint16_t)(w4[j] >> 16));
      }
#pragma unroll
      for (int h = 0; h < kMaxGroup; ++h) {
        if ((uint32_t)h < g) {
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[h] += kf[j] * qs[h][d + j];
        }
      }
    }
#pragma unroll
    for (int h = 0; h < kMaxGroup; ++h)
      if ((uint32_t)h < g) ps[h][tid] = acc[h];
  }
  __syncthreads();
  // softmax partials per head: wave w reduces heads w, w+4, ...
  for (uint32_t h = wave; h < g; h += 4) {
    float m = -INFINITY;
    for (uint32_t t = lane; t < nt; t += 64) m = fmaxf(m, ps[h][t]);
    m = wave_max(m);
    float l = 0.f;
    for (uint32_t t = lane; t < nt; t += 64) {
      const float p = __expf(ps[h][t] - m);
      ps[h][t] = p;
      l += p;
    }
    l = wave_sum(l);
    if (lane == 0) {
      ms[h] = m;
      ls[h] = l;
    }
  }
  __syncthreads();
  // P.V: lane = pair of head dims, wave = quarter of the tokens
  const uint32_t d0 = lane * 2;
  float o0[kMaxGroup], o1[kMaxGroup];
#pragma unroll
  for (int h = 0; h < kMaxGroup; ++h) o0[h] = o1[h] = 0.f;
  if (d0 < a.hd) {
    for (uint32_t t = wave; t < nt; t += 4) {
      const uint32_t vv = *reinterpret_cast<const uint32_t*>(vbase + (uint64_t)(t0 + t) * a.hd + d0);
      const float v0 = dbf((uint16_t)vv), v1 = dbf((uint16_t)(vv >> 16));
#pragma unroll
      for (int h = 0; h < kMaxGroup; ++h) {
        if ((uint32_t)h < g) {
          const float p = ps[h][t];
          o0[h] += p * v0;
          o1[h] += p * v1;
        }
      }
    }
#pragma unroll
    for (int h = 0; h < kMaxGroup; ++h)
      if ((uint32_t)h < g) {
        part[wave][h][d0] = o0[h];
        part[wave][h][d0 + 1] = o1[h];
      }
  }
  __syncthreads();
  // reduce the 4 waves and store this split's partial (unnormalised) + m, l
  for (uint32_t e = tid; e < g * a.hd; e += 256) {
    const uint32_t h = e / a.hd, d = e - h * a.hd;
    const float o = part[0][h][d] + part[1][h][d] + part[2][h][d] + part[3][h][d];
    const uint64_t row = ((uint64_t)b * a.hq + kvh * g + h) * a.nsplit + split;
    a.part_o[row * a.hd + d] = o;
    if (d == 0) {
      a.part_ml[row * 2] = ms[h];
      a.part_ml[row * 2 + 1] = ls[h];
    }
  }
}

// Wave-split decode attention on the matrix cores (the default for hd 64 / 128).
// The workgroup's 256 tokens are four independent 64-token runs, one per wave:
// no block-wide barrier sits between the phases, and LDS holds only the
// probabilities and the four wave partials (24 KB for a group of 8 - the lane-
// per-token kernel above needs 56 KB: 2 workgroups per CU).
//  * Q.K is a [64 tokens x hd] . [hd x 16 heads] GEMM per wave on
//    v_mfma_f32_16x16x32_bf16: the A fragment of a 16-token tile is one 16 B
//    load per lane straight from the K rows (lane l: token l&15, dims
//    8(l>>4)..+8 of the 32-dim step - every load a fully used 1 KB wave
//    access), B is the query group (heads padded to 16), and all 16 (hd 128)
//    K fragments are in flight before the first MFMA.
//  * D lands as lane l = head l&15, tokens 4(l>>4)+r of each tile: the softmax
//    max / sum over a head's 64 tokens is a 16-value local reduction plus two
//    xor shuffles for ALL heads at once (the lane-per-token kernel shuffles per
//    head).
//  * P.V (contraction over tokens, V rows are dim-contiguous) stays on the
//    vector ALUs: half a wave per token, 4 dims per lane, p broadcast from LDS.
// The four wave partials are merged (log-sum-exp) into the split partial the
// combine kernel reads (same part_o / part_ml layout as k_attn_decode).
typedef __bf16 attn_bf16x8_t __attribute__((ext_vector_type(8)));
typedef float attn_f32x4_t __attribute__((ext_vector_type(4)));

// Variants (OGKM_ATTN_VAR, A/B drills): TH4 - all four K tiles in flight at
// once; EV - the first V round is requested before the softmax.
template <int HD, int G, int NW, int DPL, bool TH4, bool EV>
__global__ void __launch_bounds__(256) k_attn_decode_ws(AttnArgs a) {
  constexpr int KS = HD / 32;         // 32-dim MFMA steps
  static_assert((HD == 64 || HD == 128) && G <= 16, "shape");
  extern __shared__ float smem[];
  const uint32_t g = a.hq / a.hkv;    // <= G
  float* ps = smem;                   // [NW waves][64 tokens][G] probabilities (token-major, G padded)
  float* po = smem + NW * G * 64;     // [NW waves][g][HD] unnormalised outputs
  __shared__ float wm[NW][G], wl[NW][G];
  const uint32_t split = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t wt0 = split * (64u * NW) + wave * 64;
  const int32_t wn = (int32_t)a.len - (int32_t)wt0 < 64 ? (int32_t)a.len - (int32_t)wt0 : 64;
  float* wps = ps + wave * G * 64;
  float* wpo = po + wave * g * HD;
  if (wn <= 0) {  // this wave's tokens are past the context: an empty partial
    for (uint32_t e = lane; e < g * HD; e += 64) wpo[e] = 0.f;
    if (lane < g) {
      wm[wave][lane] = -INFINITY;
      wl[wave][lane] = 0.f;
    }
  } else {
    const uint16_t* kbase = a.cache + ((uint64_t)b * a.hkv + kvh) * (uint64_t)a.T * HD;
    const uint16_t* vbase = a.cache + (((uint64_t)a.B + b) * a.hkv + kvh) * (uint64_t)a.T * HD;
    const uint32_t col = lane & 15, quad = lane >> 4;
    // B fragments: the query group, head `col` (zero past the group)
    uint4 qb[KS];
    const uint16_t* qr = a.q + ((uint64_t)b * a.hq + kvh * g + (col < g ? col : 0)) * HD + 8 * quad;
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      qb[k] = *reinterpret_cast<const uint4*>(qr + 32 * k);
      if (col >= g) qb[k] = uint4{0u, 0u, 0u, 0u};
    }
    // A fragments: 4 token tiles x KS dim steps, two tiles' loads in flight at a
    // time for big groups (the P.V accumulators need the registers), all four
    // for small ones (rows past the context are clamped and masked below)
    constexpr int TH = TH4 ? 4 : 2;
    attn_f32x4_t sc[4];
#pragma unroll 1
    for (int t0 = 0; t0 < 4; t0 += TH) {
      uint4 ka[TH][KS];
#pragma unroll
      for (int t = 0; t < TH; ++t) {
        const int32_t tok = (t0 + t) * 16 + (int32_t)col;
        const uint32_t row = wt0 + (uint32_t)(tok < wn ? tok : wn - 1);
        const uint16_t* kr = kbase + (uint64_t)row * HD + 8 * quad;
#pragma unroll
        for (int k = 0; k < KS; ++k) ka[t][k] = *reinterpret_cast<const uint4*>(kr + 32 * k);
      }
#pragma unroll
      for (int t = 0; t < TH; ++t) {
        attn_f32x4_t acc = attn_f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < KS; ++k)
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(attn_bf16x8_t, ka[t][k]),
                                                        __builtin_bit_cast(attn_bf16x8_t, qb[k]), acc, 0, 0, 0);
        sc[t0 + t] = acc;
      }
    }
    // P.V geometry (see below)
    static_assert(DPL == 8 || DPL == 4, "dims per lane");
    constexpr int LPT = HD / DPL, TPI = 64 / LPT, NI = 64 / TPI;
    constexpr int VB = 8;
    const uint32_t tg = lane / LPT, dg = lane % LPT;
    const uint16_t* vcol = vbase + (uint64_t)wt0 * HD + dg * DPL;
    uint32_t vv[VB][DPL / 2];
    auto load_v = [&](int i0) {
#pragma unroll
      for (int i = 0; i < VB; ++i) {
        const int32_t t = (i0 + i) * TPI + (int32_t)tg;
        const int32_t tt = t < wn ? t : wn - 1;  // past the context: clamped, its p is 0
        if constexpr (DPL == 8) {
          const uint4 w = *reinterpret_cast<const uint4*>(vcol + (uint64_t)tt * HD);
          vv[i][0] = w.x;
          vv[i][1] = w.y;
          vv[i][2] = w.z;
          vv[i][3] = w.w;
        } else {
          const uint2 w = *reinterpret_cast<const uint2*>(vcol + (uint64_t)tt * HD);
          vv[i][0] = w.x;
          vv[i][1] = w.y;
        }
      }
    };
    if constexpr (EV) load_v(0);  // the first V round flies during the softmax
    // softmax partials: lane = head col, tokens t*16 + 4*quad + r
    float m = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int32_t tok = t * 16 + 4 * (int32_t)quad + r;
        const float v = tok < wn ? sc[t][r] * a.scale : -INFINITY;
        sc[t][r] = v;
        m = fmaxf(m, v);
      }
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float l = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = __expf(sc[t][r] - m);  // masked tokens: exp(-inf) = 0
        l += p;
        if (col < G) wps[(t * 16 + 4 * quad + r) * G + col] = col < g ? p : 0.f;
      }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    if (quad == 0 && col < g) {
      wm[wave][col] = m;
      wl[wave][col] = l;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    // P.V on the vector ALUs, bound by how many V bytes are in flight: lane l
    // owns DPL dims (dim group l % LPT) of every TPI-th token (token group
    // l / LPT); one wave instruction loads TPI whole V rows and VB of them are
    // issued before the first FMA (8 KB per wave for G <= 8 - the
    // half-wave-per-token loop had 2 KB in flight and capped the tp8 shape,
    // one KV head per batch row, at ~1.3 TB/s). The token groups' partial
    // sums are reduced with xor shuffles at the end.
    // DPL dims per lane (template): 8 - one 16 B load per row piece (groups of
    // up to 4 heads); 4 - 96 VGPRs and four waves per SIMD for 8 and 16 heads.
    float o[G][DPL];
#pragma unroll
    for (int h = 0; h < G; ++h)
#pragma unroll
      for (int j = 0; j < DPL; ++j) o[h][j] = 0.f;
#pragma unroll 1
    for (int i0 = 0; i0 < NI; i0 += VB) {
      if (!EV || i0) load_v(i0);
#pragma unroll
      for (int i = 0; i < VB; ++i) {
        const int32_t t = (i0 + i) * TPI + (int32_t)tg;
        float vf[DPL];
#pragma unroll
        for (int j = 0; j < DPL / 2; ++j) {
          vf[2 * j] = dbf((uint16_t)vv[i][j]);
          vf[2 * j + 1] = dbf((uint16_t)(vv[i][j] >> 16));
        }
        const float* pt = wps + t * G;  // token-major probabilities, G (padded) heads
#pragma unroll
        for (int h = 0; h < G; ++h) {
          const float p = pt[h];
#pragma unroll
          for (int j = 0; j < DPL; ++j) o[h][j] += p * vf[j];
        }
      }
    }
#pragma unroll
    for (int h = 0; h < G; ++h) {
#pragma unroll
      for (int j = 0; j < DPL; ++j) {
        float x = o[h][j];
#pragma unroll
        for (int sh = LPT; sh < 64; sh <<= 1) x += __shfl_xor(x, sh, 64);
        if (tg == 0 && (uint32_t)h < g) wpo[h * HD + dg * DPL + j] = x;
      }
    }
  }
  __syncthreads();
  // merge the NW wave partials into this split's partial
  for (uint32_t e = threadIdx.x; e < g * HD; e += 64 * NW) {
    const uint32_t h = e / HD, d = e - h * HD;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < NW; ++w) M = fmaxf(M, wm[w][h]);
    float acc = 0.f, l = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const float f = wm[w][h] == -INFINITY ? 0.f : __expf(wm[w][h] - M);
      acc += f * po[(w * g + h) * HD + d];
      l += f * wl[w][h];
    }
    const uint64_t row = ((uint64_t)b * a.hq + kvh * g + h) * a.nsplit + split;
    a.part_o[row * HD + d] = acc;
    if (d == 0) {
      a.part_ml[row * 2] = M;
      a.part_ml[row * 2 + 1] = l;
    }
  }
}

// One workgroup of hd threads per (b, q head): merge the splits. Splits are
// read 8 at a time, all loads of a group issued before the first use (one
// dependent memory round per 8 splits instead of two passes over them), with
// the running max rescaling the sums between groups; up to 8 splits (2048
// tokens) the arithmetic is exactly the two-pass merge's.
__global__ void k_attn_combine(AttnArgs a) {
  const uint32_t bh = blockIdx.x;  // b * hq + h
  const uint32_t d = threadIdx.x;
  const uint64_t r0 = (uint64_t)bh * a.nsplit;
  float M = -INFINITY, num = 0.f, den = 0.f;
  for (uint32_t s0 = 0; s0 < a.nsplit; s0 += 8) {
    float m[8], l[8], o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint64_t row = r0 + (s0 + j < a.nsplit ? s0 + j : a.nsplit - 1);  // clamped: masked below
      m[j] = a.part_ml[row * 2];
      l[j] = a.part_ml[row * 2 + 1];
      o[j] = d < a.hd ? a.part_o[row * a.hd + d] : 0.f;
    }
    float mb = M;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (s0 + j < a.nsplit) mb = fmaxf(mb, m[j]);
    if (M != -INFINITY) {  // earlier groups' sums, rescaled to the new max
      const float sc = __expf(M - mb);
      num *= sc;
      den *= sc;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (s0 + j < a.nsplit) {
        const float w = __expf(m[j] - mb);
        den += w * l[j];
        num += w * o[j];
      }
    M = mb;
  }
  if (d < a.hd) {
    const uint32_t b = bh / a.hq, col = (bh - b * a.hq) * a.hd + d;
    a.out[a.out_frag ? frag_index(b, col, a.hq * a.hd) : (uint64_t)bh * a.hd + d] = df2bf(num / den);
  }
}

hipError_t launch_rmsnorm(const ResidNormArgs& a, hipStream_t s) {
  if (a.dim % 4 || a.dim < 4 || a.dim > 16 * kNormCols || a.ldx % 4 || a.ldy % 4 || (a.y_frag && a.dim % 32))
    return hipErrorInvalidValue;
  if (!a.rows) return hipSuccess;
  // Few rows: two wide launches (every 1024-column block its own workgroup).
  if (a.ssq && a.rows < kNormWideRows) {
    const dim3 grid((a.dim + kNormCols - 1) / kNormCols, a.rows);
    hipLaunchKernelGGL(k_norm_ssq, grid, dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_norm_scale, grid, dim3(256), 0, s, a);
    return hipGetLastError();
  }
  static const bool wide1k = !getenv("OGKM_NORM_1K") || atoi(getenv("OGKM_NORM_1K")) != 0;
  if (wide1k && a.rows < kNormWideRows && a.dim > kNormCols && a.dim <= 8 * kNormCols) {
    if (a.dim <= 4 * kNormCols)
      hipLaunchKernelGGL((k_rmsnorm<1, 1024>), dim3(a.rows), dim3(1024), 0, s, a);
    else
      hipLaunchKernelGGL((k_rmsnorm<2, 1024>), dim3(a.rows), dim3(1024), 0, s, a);
    return hipGetLastError();
  }
  if (a.dim <= kNormCols)
    hipLaunchKernelGGL((k_rmsnorm<1>), dim3(a.rows), dim3(256), 0, s, a);
  else if (a.dim <= 4 * kNormCols)
    hipLaunchKernelGGL((k_rmsnorm<4>), dim3(a.rows), dim3(256), 0, s, a);
  else if (a.dim <= 8 * kNormCols)
    hipLaunchKernelGGL((k_rmsnorm<8>), dim3(a.rows), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((k_rmsnorm<16>), dim3(a.rows), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_rope_kv(const RopeKvArgs& a, hipStream_t s) {
  if (a.hd % 2 || a.pos >= a.T || (a.tail && a.tail_pos >= a.tail_T)) return hipErrorInvalidValue;
  const uint64_t n = (uint64_t)a.B * (a.hq + 2 * a.hkv) * (a.hd / 2);
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_rope_kv, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_attn_decode(AttnArgs a, hipStream_t s) {
  if (!a.hkv || a.hq % a.hkv || a.hq / a.hkv > (uint32_t)kMaxGroup || a.hd > (uint32_t)kMaxHd || a.hd % 8 ||
      !a.len || a.len > a.T)
    return hipErrorInvalidValue;
  const bool ws = a.hd == 128 || a.hd == 64;
  const uint32_t st = ws ? a.split_tokens : (uint32_t)kAttnSplit;
  if ((st != 64 && st != 256) || a.nsplit != (a.len + st - 1) / st) return hipErrorInvalidValue;
  if (a.out_frag && (a.hq * a.hd) % 32) return hipErrorInvalidValue;
  const uint32_t g = a.hq / a.hkv;
  const uint32_t gg = g <= 4 ? 4 : g <= 8 ? 8 : 16;
  const dim3 grid(a.nsplit, a.hkv, a.B);
  const uint32_t nw = st / 64;
  const size_t lds = (size_t)nw * (gg * 64 + g * a.hd) * sizeof(float);  // token-major p (G padded) + outputs
  if (ws) {
#define OGKM_ATTN_WS(HD, L, NW, D)                                                                      \
  do switch (var) {                                                                                    \
    case 1: hipLaunchKernelGGL((k_attn_decode_ws<HD, L, NW, D, true, false>), grid, dim3(64 * NW), lds, s, a); break; \
    case 2: hipLaunchKernelGGL((k_attn_decode_ws<HD, L, NW, D, false, true>), grid, dim3(64 * NW), lds, s, a); break; \
    case 3: hipLaunchKernelGGL((k_attn_decode_ws<HD, L, NW, D, true, true>), grid, dim3(64 * NW), lds, s, a); break;  \
    case 0: hipLaunchKernelGGL((k_attn_decode_ws<HD, L, NW, D, false, false>), grid, dim3(64 * NW), lds, s, a); break; \
    default: hipLaunchKernelGGL((k_attn_decode_ws<HD, L, NW, D, false, true>), grid, dim3(64 * NW), lds, s, a);       \
  } while (0)
    // groups of 8: 4 dims per lane at every measured shape (70B tp8 1.56 vs 1.42 TB/s with 8,
    // 70B 3.76 vs 2.70; gpurun_out/r5/g_attn_dpl*.log); OGKM_ATTN_DPL=8 for A/B drills
    static const int force_dpl = getenv("OGKM_ATTN_DPL") ? atoi(getenv("OGKM_ATTN_DPL")) : 0;
    const bool wide = force_dpl == 8;
    // early V by default: faster at every measured shape (graph-timed, MALL-cold;
    // 8B 4.14 vs 4.04, 70B 4.04 vs 3.78, 70B-tp8 1.72 vs 1.58, 405B-tp8 1.33 vs
    // 1.25 TB/s; profiles/r5_attn_variants.txt); OGKM_ATTN_VAR=0..3 for A/B drills
    static const int var = getenv("OGKM_ATTN_VAR") ? atoi(getenv("OGKM_ATTN_VAR")) : 2;
#define OGKM_ATTN_WS_G(HD, NW)                      \
  if (gg == 4) OGKM_ATTN_WS(HD, 4, NW, 8);          \
  else if (gg == 8 && wide) OGKM_ATTN_WS(HD, 8, NW, 8); \
  else if (gg == 8) OGKM_ATTN_WS(HD, 8, NW, 4);     \
  else OGKM_ATTN_WS(HD, 16, NW, 4)
    if (a.hd == 128) {
      if (nw == 1) { OGKM_ATTN_WS_G(128, 1); } else { OGKM_ATTN_WS_G(128, 4); }
    } else {
      if (nw == 1) { OGKM_ATTN_WS_G(64, 1); } else { OGKM_ATTN_WS_G(64, 4); }
    }
#undef OGKM_ATTN_WS_G
#undef OGKM_ATTN_WS
  } else {
    hipLaunchKernelGGL(k_attn_decode, grid, dim3(256), 0, s, a);
  }
  hipLaunchKernelGGL(k_attn_combine, dim3(a.B * a.hq), dim3(a.hd < 64 ? 64 : a.hd), 0, s, a);
  return hipGetLastError();
}

}  // namespace ogkm
