// Decode-GEMM argument blocks shared by the HIP kernels (decode_gemm.hip), the
// backends (HIP launch / fake CPU reference) and the bindings. No HIP headers.
#pragma once

#include <cstdint>

namespace ogkm {

enum DGemmEpilogue : uint32_t { DGEMM_EPI_STORE = 0, DGEMM_EPI_RESID = 1, DGEMM_EPI_SILU_MUL = 2 };
struct DGemmReduceArgs {
  const float* part;
  uint32_t ksplit, M, N;   // N = columns of part (SILU_MUL: 2 f, gate then up)
  uint32_t epi;
  const uint16_t* resid;   // RESID: bf16 [M, ldr]
  uint32_t ldr, ldo;
  uint16_t* out;           // bf16 [M, ldo] (may alias resid)
  uint32_t out_frag;       // 1: out is fragment-ordered [M16][out_cols]; this launch writes columns
  uint32_t out_cols, out_col0;  // out_col0 .. out_col0 + nout of it (ldo unused)
};
// Decode GEMM (csrc/kernels/decode_gemm.hip): part[ks][M][N] = X[M,K] . W[N,K]^T
// over K split `ks`, with W in fragment order (16x32 MFMA A-tiles, 1 KB each)
// either as raw bf16 or inside a BF11/raw packed stream (decoded in registers).
struct DGemmArgs {
  const uint8_t* w;       // raw: bf16 fragment-ordered weights; packed: stream base
  uint64_t w_off;         // value offset of this tensor (raw: from w; packed: in the stream's value space)
  const uint16_t* x;      // [M, K] bf16, row stride ldx (elements, multiple of 8)
  float* part;            // [ksplit][M][N] f32
  uint32_t M, N, K, ldx;
  uint32_t ksplit, klen;  // K range per split (multiple of 32)
  uint32_t row_blocks;    // ceil(N / 64)
  uint32_t chunk_shift;   // packed: log2(stream chunk_values)
  uint32_t unroll;        // K steps per pipelined block (1, 2 or 4; 0 = default)
  uint32_t lds_x;         // raw weights: 1 = row tile per wave, activations shared through LDS
  uint32_t wg_waves;      // split-K kernels: waves per workgroup (0 / 4 = 256 threads, 1 = one-wave
                          // workgroups, so a few hundred units spread over every CU)
  uint32_t depth;         // pipelined raw kernel: 0 / 4 = k_dgemm_pipe (two register sets of 2 K
                          // steps), 10 D = k_dgemm_lring (LDS ring of D K steps, D = 3..7)
  uint32_t x_frag;        // 1: x is fragment-ordered (frag_index below; rows padded to 16, ldx unused)
  // In-kernel split-K fixup (k_dgemm_pipe / k_dgemm_lring): when set, every
  // wave counts its arrival on its output group's counter (agent-scope
  // atomic between release / acquire fences); the last of the group's
  // ksplit (SILU_MUL: 2 ksplit - the gate and up row blocks) sums the splits
  // and applies `fix`'s epilogue - no k_dgemm_reduce launch. Counters are
  // zero between launches (the last arrival resets its own); one slab per
  // stream. Group = row block (SILU_MUL: row block mod row_blocks / 2,
  // needs (N / 2) % 64 == 0); index blockIdx.y * row_blocks + group.
  uint32_t* fix_cnt;
  DGemmReduceArgs fix;
  // One K split, STORE / RESID epilogue (same kernels): every wave writes
  // `fix`'s epilogue from its accumulators - no partials, no reduce launch.
  uint32_t direct;
};

// Fragment order of an [M, K] bf16 activation (K % 32 == 0, M padded to a
// multiple of 16): 16 x 32 tiles, tile (m / 16, k / 32) at index
// (m / 16) * (K / 32) + k / 32, 1 KB each, lane-major - the B-operand fragment
// of v_mfma_f32_16x16x32_bf16, exactly as the weights are stored. A GEMM wave
// then fetches each activation fragment with one contiguous 1 KB access (8
// full cache lines) instead of 16 half-lines; the producers (RMSNorm, the
// attention combine, the SiLU-mul epilogue) write this order directly.
// Elements k .. k + 3 (k % 4 == 0) of one row are contiguous.
constexpr uint64_t frag_index(uint32_t m, uint32_t k, uint32_t K) {
  return ((((uint64_t)(m >> 4) * (K >> 5) + (k >> 5)) * 64u + (m & 15u) + 16u * ((k >> 3) & 3u)) << 3) + (k & 7u);
}
// Weight source: raw bf16 fragments; a packed stream with BF11 and raw chunks;
// a packed stream whose chunks are all BF11 (fast, phase-pipelined path).
enum DGemmWeights : int { DGEMM_W_RAW = 0, DGEMM_W_PACKED = 1, DGEMM_W_PACKED_BF11 = 2 };
// The fixup runs in the pipelined raw kernels only (k_dgemm_pipe /
// k_dgemm_lring: raw weights, unroll 1, no LDS-x), with `fix` describing the
// same partial slab; SILU_MUL pairs gate row block g with up row block
// g + row_blocks / 2, so the halves must be whole 64-row blocks.
inline bool dgemm_fixup_ok(const DGemmArgs& a, int mode) {
  if (mode != DGEMM_W_RAW || a.unroll != 1 || a.lds_x) return false;
  if (a.fix.part != a.part || a.fix.ksplit != a.ksplit || a.fix.M != a.M || a.fix.N != a.N) return false;
  return a.fix.epi != DGEMM_EPI_SILU_MUL || (a.N / 2) % 64 == 0;
}
// Split-K plan: enough waves to fill the chip (>= ~4 per CU over 256 CUs) while
// keeping each split's K range a multiple of 32.
inline void dgemm_plan(uint32_t N, uint32_t K, uint32_t target_units, uint32_t* ksplit, uint32_t* klen) {
  const uint32_t rb = (N / 16 + 3) / 4;
  uint32_t ks = rb >= target_units ? 1 : (target_units + rb - 1) / rb;
  const uint32_t ksteps = K / 32;
  const uint32_t max_ks = ksteps / 4 ? ksteps / 4 : 1;  // >= 128 of K per split
  if (ks > max_ks) ks = max_ks;
  uint32_t steps = (ksteps + ks - 1) / ks;
  *klen = steps * 32;
  *ksplit = (K + *klen - 1) / *klen;
}

// ---- fused decode-step ops (csrc/kernels/decode_ops.hip)
// KV cache layout: [2][B][Hkv][T][hd] bf16 (k then v).
struct RopeKvArgs {
  const uint16_t* qkv;     // [B, (hq + 2 hkv) * hd], row stride ldqkv
  uint32_t ldqkv;
  const float* cos;        // [hd / 2] at this position
  const float* sin;
  uint16_t* q_out;         // [B, hq, hd] rotated q
  uint16_t* cache;         // [2][B][hkv][T][hd]: rotated k and v written at `pos`
  uint16_t* tail;          // optional second copy [2][B][hkv][tail_T][hd] at `tail_pos`
  uint32_t B, hq, hkv, hd, T, pos, tail_T, tail_pos;
  // Deferred qkv GEMM: when set, qkv is bf16(sum over ksplit of part[k][B][N])
  // (N = (hq + 2 hkv) hd, the decode GEMM's store epilogue) and `qkv` is unused.
  const float* part;
  uint32_t ksplit;
};
// RMSNorm over `rows` rows of x, optionally after the deferred residual GEMM
// epilogue: with part set, x += bf16(sum over ksplit of part[k][rows][dim])
// (x updated in place, = k_dgemm_reduce's RESID epilogue), then
// y = bf16(bf16(x * rsqrt(mean(x^2) + eps)) * w).
struct ResidNormArgs {
  const float* part;       // nullptr: plain RMSNorm
  uint32_t ksplit;
  uint16_t* x;             // [rows, ldx] bf16
  const uint16_t* w;       // [dim]
  uint16_t* y;             // [rows, ldy] (y_frag: fragment-ordered [rows16][dim], ldy unused)
  uint32_t rows, dim, ldx, ldy;
  float eps;
  uint32_t y_frag;
  // Optional [rows][ceil(dim / kNormCols)] f32 scratch: with it, few-row norms
  // run as two wide launches (residual + partial sums of squares over every
  // 1024-column block, then the scaling) instead of one workgroup per row.
  float* ssq = nullptr;
};
constexpr uint32_t kNormCols = 1024;  // RMSNorm columns per pass of a 256-thread workgroup (4 per thread)
constexpr uint32_t kNormWideRows = 256;  // with an ssq scratch, norms of fewer rows take the two-launch path
struct AttnArgs {
  const uint16_t* q;       // [B, hq, hd] (rotated)
  const uint16_t* cache;   // [2][B][hkv][T][hd]
  uint16_t* out;           // [B, hq * hd]
  float* part_o;           // [B * hq * nsplit, hd] split partials (f32)
  float* part_ml;          // [B * hq * nsplit, 2]  (max, sum) per split
  uint32_t B, hq, hkv, hd, T, len, nsplit;
  float scale;
  uint32_t out_frag;       // 1: out is fragment-ordered [B16][hq * hd]
  uint32_t split_tokens;   // context tokens per workgroup: 256 (4 waves, default) or 64 (1 wave; hd 64 / 128 -
                           // measured slower at every bench shape, kept as an explicit option)
};
constexpr uint32_t kAttnSplitTokens = 256;
// CPU references of the decode-step ops (fake backend, tests).
void rmsnorm_cpu(const ResidNormArgs& a);
void rope_kv_cpu(const RopeKvArgs& a);
void attn_decode_cpu(const AttnArgs& a);

// CPU reference of k_dgemm / k_dgemm_reduce (fake backend, tests).
void dgemm_cpu(const DGemmArgs& a, bool packed);
void dgemm_reduce_cpu(const DGemmReduceArgs& a);

}  // namespace ogkm
