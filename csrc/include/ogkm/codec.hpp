// BF12: lossless packed-bf16 format for the host / CXL tiers.
//
// Streaming decode at 2x oversubscription is bound by PCIe bytes, so the host
// copy of a bf16 weight block is stored packed and the H2D copy kernel decodes
// it on the fly (csrc/kernels/bf12_kernels.hip): fewer bytes on the link, the
// exact same bf16 bits in HBM.
//
// A bf16 value is s(1) e(8) m(7). Weights cluster in a narrow exponent band, so
// per 2 MB block we pick a base exponent and store
//   sm byte    = s << 7 | m                        (1 byte / value)
//   code       = e - base  if 0 <= e - base < 15   (4 bits / value)
//              = 15        otherwise (escape: exact value in the exception list)
// Layout of one encoded block (all offsets from the block start):
//   [0, 256)                  Bf12Header
//   [256, 256 + n)            sm bytes
//   [256 + n, 256 + 1.5 n)    code nibbles (value 2i in the low nibble of byte i)
//   [256 + 1.5 n, ...)        exceptions {u32 index, u16 bits, u16 pad}, grouped by
//                             32768-value tile (tile t owns [exc_off[t], exc_off[t+1]))
// 12 bits/value + 8 B per exception: 0.75x for typical weights. A block whose
// encoding would not fit 2 MB is stored raw (Bf12 returns false).
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace ogkm {

constexpr uint32_t kBf12Magic = 0x32314642;  // "BF12"
constexpr uint32_t kBf12Tile = 32768;        // values per decode tile (64 KB of bf16)
constexpr uint32_t kBf12MaxTiles = 32;       // 2 MB block / 64 KB
constexpr uint32_t kBf12HeaderBytes = 256;

struct Bf12Header {
  uint32_t magic;
  uint32_t base;       // exponent of code 0
  uint32_t n_values;
  uint32_t n_exc;
  uint32_t exc_off[kBf12MaxTiles + 1];
  uint32_t reserved[(kBf12HeaderBytes / 4) - 4 - (kBf12MaxTiles + 1)];
};
static_assert(sizeof(Bf12Header) == kBf12HeaderBytes, "BF12 header is 256 bytes");

struct Bf12Exception {
  uint32_t index;
  uint16_t bits;
  uint16_t pad;
};

inline uint64_t bf12_encoded_bytes(uint32_t n_values, uint32_t n_exc) {
  return kBf12HeaderBytes + (uint64_t)n_values + (uint64_t)n_values / 2 + (uint64_t)n_exc * sizeof(Bf12Exception);
}

// BF11: two-level exponent code, ~11 bits/value for weight-like data (a
// Gaussian's exponent carries ~2.5 bits of entropy; BF12 spends 4).
//   sm byte       = s << 7 | m                                     (8 bits / value)
//   primary code  = index of e in prim[0..2]; 3 = escape           (2 bits / value)
//   secondary     = e - sec_base for escaped values, 15 = exception (4 bits / escape)
// With the three most frequent exponents primary, ~24% of Gaussian values
// escape: 8 + 2 + 0.24 * 4 ~= 11 bits (0.69x). The secondary nibbles of a block
// are stored in value order; a 512-value wave group (one wave, 8 values per lane)
// finds its first nibble from a per-tile base + a u16 per group, and each lane
// its own from a wave prefix count of escapes (4 ballots + mbcnt on gfx950), so
// every value decodes at a fixed cost with no serial dependency.
// Layout (offsets from the block start, recorded in the header):
//   [0, 512)            Bf11Header
//   off_prim            n/4 bytes of 2-bit codes (value i in bits 2(i%4) of byte i/4)
//   off_wg              u32 per 512-value group: its first secondary nibble (absolute)
//   off_sec             secondary nibbles (value order, low nibble first) + 8 B pad
//   off_exc             Bf12Exception list grouped by 32768-value tile
// The sm plane sits right after the header at 512.
constexpr uint32_t kBf11Magic = 0x31314642;  // "BF11"
constexpr uint32_t kBf11HeaderBytes = 512;
constexpr uint32_t kBf11Group = 512;         // values per wave group (64 lanes x 8)
struct Bf11Header {
  uint32_t magic;
  uint32_t n_values;
  uint32_t n_exc;
  uint32_t prim;       // exponents of primary codes 0..2 in bytes 0..2
  uint32_t sec_base;   // exponent of secondary code 0
  uint32_t n_sec;      // secondary nibbles
  uint32_t off_prim, off_wg, off_sec, off_exc;
  uint32_t exc_off[kBf12MaxTiles + 1];
  uint32_t sec_tile[kBf12MaxTiles + 1];
  uint32_t reserved[(kBf11HeaderBytes / 4) - 10 - 2 * (kBf12MaxTiles + 1)];
};
static_assert(sizeof(Bf11Header) == kBf11HeaderBytes, "BF11 header is 512 bytes");

// Plane offsets are a pure function of n_values (readers may compute them
// instead of loading them from the header: the decode GEMM does, to keep its
// scalar-load chain short). Only off_exc depends on the data.
#ifdef __HIPCC__
#define OGKM_HD __host__ __device__
#else
#define OGKM_HD
#endif
struct Bf11Layout {
  uint32_t off_prim, off_wg, off_sec;
};
OGKM_HD inline Bf11Layout bf11_layout(uint32_t n) {
  Bf11Layout l;
  l.off_prim = kBf11HeaderBytes + n;
  l.off_wg = (l.off_prim + n / 4 + 7u) & ~7u;
  l.off_sec = (l.off_wg + 4u * ((n + kBf11Group - 1) / kBf11Group) + 7u) & ~7u;
  return l;
}

// Encode n_values bf16 (n_values a multiple of 8, <= 1 Mi) as a BF11 block.
// Returns the encoded size, or 0 when it does not fit `cap`.
uint64_t bf11_encode(const uint16_t* in, uint32_t n_values, uint8_t* out, uint64_t cap);
bool bf11_decode(const uint8_t* in, uint16_t* out, uint32_t n_values);
// Decode the 512-value wave group starting at value v (a multiple of 512) of a
// BF11 block, exceptions included (the decode-GEMM fragment path).
void bf11_decode_group(const uint8_t* in, uint32_t v, uint16_t* out512);

// ANS1: entropy-coded exponents (interleaved rANS), sign|mantissa bytes raw.
// BF11's fixed-width codes spend ~3.1 bits on an exponent whose entropy is
// ~2.55 bits for weight-like (bell-shaped) data; rANS gets within ~0.01 bit of
// the entropy, so a value costs ~8 + 2.56 bits + segment overhead (~0.1 bit).
// Exponent-only modelling (like DFloat11-style codecs): no assumption about the
// mantissa. A chunk (<= 1 Mi values, a multiple of 512) holds:
//   [0, 1024)              AnsHeader (u16 freq[256] at byte 512: the chunk's
//                          exponent histogram normalised to 2^12)
//   [1024, 1024 + n)       sign|mantissa plane
//   off_dir (4-aligned)    u32 seg_off[n_seg + 1] (offsets from the chunk start)
//   segment s (4-aligned)  u32 state[64] + u16 words[] (renormalisation stream)
// A segment is 32 Ki values decoded by ONE wave: at step t lane l decodes
// value ((t / 8) * 64 + l) * 8 + t % 8 of the segment (so each lane assembles
// one 16-B fragment every 8 steps). rANS: 32-bit state in [2^16, 2^32), 12-bit
// precision, 16-bit renormalisation; the words of a segment are consumed in
// (step, lane) order - a wave finds each lane's word with a ballot prefix.
constexpr uint32_t kAnsMagic = 0x31534E41;  // "ANS1"
constexpr uint32_t kAnsHeaderBytes = 1024;
constexpr uint32_t kAnsSegValues = 32768;
constexpr uint32_t kAnsPrecBits = 12;
constexpr uint32_t kAnsLowBound = 1u << 16;
struct AnsHeader {
  uint32_t magic;
  uint32_t n_values;
  uint32_t n_seg;
  uint32_t off_dir;
  uint32_t reserved[124];
  uint16_t freq[256];
};
static_assert(sizeof(AnsHeader) == kAnsHeaderBytes, "ANS header is 1 KB");
// Encode n_values bf16 (a multiple of 512, <= 1 Mi) as an ANS1 chunk; 0 when
// it does not fit `cap` (the caller stores the chunk raw).
uint64_t ans_encode(const uint16_t* in, uint32_t n_values, uint8_t* out, uint64_t cap);
bool ans_decode(const uint8_t* in, uint16_t* out, uint32_t n_values);

// Decode a block stored in residency format `fmt` (1 BF12, 2 ANS1) into
// n_values 16-bit values.
bool block_decode(uint8_t fmt, const uint8_t* in, uint16_t* out, uint32_t n_values);

// Encode n_values bf16 (n_values even) into `out` (capacity `cap` bytes).
// Returns the encoded size, or 0 when the block does not compress into `cap`.
uint64_t bf12_encode(const uint16_t* in, uint32_t n_values, uint8_t* out, uint64_t cap);
// Decode an encoded block into n_values bf16.
bool bf12_decode(const uint8_t* in, uint16_t* out, uint32_t n_values);

// BF12 stream: a whole tensor kept packed in ANY tier, HBM included (the
// weights of a tiered model stay packed where they rest and are unpacked into a
// bf16 staging buffer right before use: k_bf12_unpack). The tensor is cut into
// chunks of `chunk_values` (a power of two, 8 Ki .. 1 Mi values); each chunk is
// a BF12 block, or raw bf16 when it does not compress / has a tail that is not
// a multiple of 8. The stream is self-describing:
//   [0, 32)            Bf12StreamHeader
//   [32, 32 + 16 n)    Bf12StreamChunk table
//   256-B aligned      chunk payloads (offsets are from the stream start)
constexpr uint32_t kBf12StreamMagic = 0x31534642;  // "BFS1"
struct Bf12StreamHeader {
  uint32_t magic;
  uint32_t nchunks;
  uint32_t chunk_values;
  uint32_t reserved;
  uint64_t n_values;
  uint64_t bytes;  // total stream size
};
struct Bf12StreamChunk {
  uint64_t offset;
  uint32_t n_values;
  uint32_t encoded;  // 0 = raw bf16, 1 = BF12 block, 2 = BF11 block
};
// BF11_STRICT: BF11 or raw only (streams read by the decode GEMM, which decodes
// those two chunk kinds in registers). ANS: ANS1 or raw chunks (encoded = 3),
// unpacked by k_ans_unpack.
enum class PackFormat : uint32_t { BF12 = 1, BF11 = 2, BF11_STRICT = 3, ANS = 4 };
static_assert(sizeof(Bf12StreamHeader) == 32 && sizeof(Bf12StreamChunk) == 16, "stream layout");
inline uint64_t bf12_stream_head_bytes(uint64_t nchunks) { return (32 + 16 * nchunks + 255) & ~255ull; }
inline uint64_t bf12_pack_bound(uint64_t n_values, uint32_t chunk_values) {
  uint64_t chunks = (n_values + chunk_values - 1) / chunk_values;
  return bf12_stream_head_bytes(chunks) + n_values * 2 + chunks * 512;
}
// Pack n_values bf16 with `threads` encoder threads into `out` (capacity >=
// bf12_pack_bound). Each chunk takes the smallest of {BF11 (when fmt is BF11),
// BF12, raw}. Returns the stream size, 0 on bad arguments.
uint64_t bf12_pack(const uint16_t* in, uint64_t n_values, uint32_t chunk_values, uint8_t* out, uint64_t cap,
                   unsigned threads, PackFormat fmt = PackFormat::BF12);
// Reference unpack of a whole stream (CPU).
// dst_stride: chunk c lands at out + c * dst_stride values (0 = contiguous).
bool bf12_unpack(const uint8_t* stream, uint16_t* out, uint64_t n_values, uint64_t dst_stride = 0,
                 uint32_t row_shift = 0);

}  // namespace ogkm
