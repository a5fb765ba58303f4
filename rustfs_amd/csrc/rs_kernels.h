// rs_kernels.h — kernel parameter blocks and launchers (internal to librsgpu).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rsg {

constexpr int kMaxC = 16;  // inputs per launch (more are chained with GF_MODE_XOR)
constexpr int kMaxR = 8;   // outputs per launch (more are split over launches)

enum GfMode : uint32_t {
    GF_MODE_STORE = 0,    // out = M * in
    GF_MODE_XOR = 1,      // out ^= M * in  (continuation of a C > 16 product)
    GF_MODE_COMPARE = 2,  // ok_flags[stripe] = 0 where out != M * in  (verify)
    // rows r < n_store: STORE at out_base + s*out_stripe_stride + out_off[r];
    // rows r >= n_store: COMPARE at out_base + s*cmp_stripe_stride + out_off[r]
    // (GET: rebuild missing data and check surplus parity in one pass)
    GF_MODE_STORE_COMPARE = 3,
};

// Launch-shape knobs for A/B measurements, resolved ONCE per process from
// the environment (rsg::tuning(), first use: rsg_create) — never read per
// call.  Production runs leave every variable unset and get the defaults
// below, which are the measured-best shapes (DESIGN.md cites the A/B runs).
// Measurement builds (`make MEASURE=1`, tools/ A/B runs): the RSG_* environment
// variables select kernels, and the A/B-only kernel variants are compiled in.
// The shipped library is built with 0.
#ifndef RSG_MEASUREMENT_BUILD
#define RSG_MEASUREMENT_BUILD 0
#endif

struct Tuning {
    bool fused = true;            // RSG_FUSED=0: encode, then a separate hash launch
    bool lost_disk_fast = true;   // RSG_LOST_DISK_FAST=0: general GET/heal order
    bool zero_copy = true;        // RSG_ZERO_COPY=0: stage pinned blocks through device memory
    int vec_block = 0;            // RSG_VEC_BLOCK=64|256: GF workgroup size for every launch (0: by layout)
    int vec_occ = -1;             // RSG_VEC_OCC=<0..8>: waves per SIMD for every GF launch (-1: default rule)
    bool rolled = false;          // RSG_ROLLED=1: rolled GF kernel for every C
    bool hash_direct_copy = false;  // RSG_HASH_COPY=1: 8-byte copy stores in the GET gather
    int hash_depth = 2;           // RSG_HASH_DEPTH=1..3: 8-packet batches in flight per lane
    int fused_kind = 0;  // RSG_FUSED_KIND=packed|ring|dma|wide2|wide4|split2|split4|net|table (0: by batch size)
    bool fused_spw1 = false;      // RSG_FUSED_SPW1=1: one stripe per packed workgroup (measurement builds; no effect in the product)
    int enc_prio = 0;             // RSG_ENC_PRIO=<0..3>: wave priorities of the fused DMA kernel
    int dma_ew = 2;               // RSG_DMA_EW=4: two encoder waves per stripe group (split, alternate steps)
    int dma_nt = 3;               // RSG_DMA_NT=<0..3>: non-temporal loads (bit 0) / stores (bit 1)
    int dma_spw = 8;              // RSG_DMA_SPW=4: four stripes per fused DMA workgroup
    int get_prio = 2;             // RSG_DMA_PRIO=<0..3>: wave priorities of the one-pass GET/heal
    bool decode_net = true;       // RSG_DECODE_NET=0: run-time-table GF waves for every one-pass pattern
    int net12_rd = 2;             // RSG_NET12_RD=4: RS(12,4) / RS(10,4) GET ring of 4 slots, one workgroup per CU
                                  // (A/B; its kernels exist in measurement builds only)
    bool hash_unal = true;        // RSG_HASH_UNAL=0: unaligned 8-byte loads for unaligned messages (A/B)
    bool get_cached = true;       // RSG_GET_CACHED=0: non-temporal output stores in the network GET/heal kernel
};
const Tuning& tuning();

// Wave-priority bits of the DMA kernels (GfApplyParams::wave_prio): bit 0
// raises the hash waves (s_setprio 2), bit 1 the GF / encoder waves.
constexpr uint32_t kPrioHash = 1, kPrioGf = 2;

// Passed by value: lands in the kernel-argument segment (SGPR-loaded).
struct GfApplyParams {
    const uint8_t* base;         // input stripe 0
    uint8_t* out_base;           // output stripe 0
    uint64_t stripe_stride;      // bytes between input stripes
    uint64_t out_stripe_stride;  // bytes between output stripes
    uint64_t in_off[kMaxC];      // byte offset of input c inside a stripe
    uint64_t out_off[kMaxR];     // byte offset of output r inside a stripe
    uint32_t tab[kMaxR][kMaxC][5];  // v_perm tables per coefficient (rs_kernels.hip)
    uint8_t* ok_flags;           // GF_MODE_COMPARE target, one byte per stripe
    uint32_t C, R, mode;
    uint32_t units;              // 16-byte units per shard (vector path)
    uint32_t chunks_per_stripe;  // set by the launcher
    uint64_t byte_begin, byte_end;  // byte path column range
    uint32_t n_store;               // GF_MODE_STORE_COMPARE split
    uint64_t cmp_stripe_stride;     // GF_MODE_STORE_COMPARE compare-row stripe stride
    // copy-through: input c with bit c of copy_mask is also stored verbatim at
    // out_base + s*out_stripe_stride + copy_off[c] (GET: the present data
    // shards are gathered by the same pass that rebuilds the missing ones)
    uint32_t copy_mask;
    uint64_t copy_off[kMaxC];
    uint32_t wave_prio;  // DMA kernels: kPrioHash | kPrioGf (set by the launcher)
    uint32_t cached_stores;  // k_decode_records_net: 1 = plain (cached) output stores instead of non-temporal
};

constexpr int kMaxHashBases = 32;

struct HashParams {
    const uint8_t* data;
    uint64_t len;            // message length
    uint64_t n;              // messages
    uint64_t shards;         // messages per stripe (1 for a plain batch)
    uint64_t shard_pitch;    // bytes between messages of one stripe
    uint64_t stripe_stride;  // bytes between stripes
    uint64_t key[4];
    uint8_t* out;            // digests (may be null in verify mode)
    uint64_t out_stride;     // bytes between digests j and j+1 (0 = 32: packed)
    // verify mode (expect != null): compare with the stored digest of message j
    // at expect + j*expect_stride and clear flags[j] on mismatch.  Callers set
    // every flag to 1 first: a multi-file verify that launch_hh256 hands to the
    // DMA-ring walk (launch_verify_records_dma, rs_verify.hip) writes each
    // flag whole (1 verified, 0 not), so a flag pre-cleared by the caller is
    // not kept
    const uint8_t* expect;
    uint64_t expect_stride;
    uint8_t* flags;
    // multi-file mode (nbases > 0): message j is record r = j % per_base of
    // file b = j / per_base, at base[b] + r*stripe_stride; its digest (stored
    // or written) sits at message + digest_off (BitrotWriter records: -32).
    // One launch then covers every shard file of a set.
    uint32_t nbases;
    uint64_t per_base;
    int64_t digest_off;
    const uint8_t* base[kMaxHashBases];
    uint8_t* flag_base[kMaxHashBases];  // verify mode with per-file flag arrays (else flags + j)
    // multi-file mode, optional: copy each message to copy_base[b] + r*copy_stride
    // while hashing it (GET: verify-before-use and gather in one pass)
    uint8_t* copy_base[kMaxHashBases];
    uint64_t copy_stride;
};

hipError_t launch_gf_apply_vec(GfApplyParams p, uint64_t n_stripes, hipStream_t stream);
hipError_t launch_gf_apply_byte(GfApplyParams p, uint64_t n_stripes, hipStream_t stream);
hipError_t launch_hh256(const HashParams& p, hipStream_t stream);
// A multi-file verify of records at unaligned pitches on the LDS-DMA ring
// (rs_verify.hip); false: not taken, launch_hh256 runs the quad kernel.
bool launch_verify_records_dma(const HashParams& h, hipStream_t stream);
// n bytes of device memory to page-locked host memory (dst = its device
// view), as a kernel on the stream; 16-byte aligned ends.
hipError_t launch_copy_to_host(uint8_t* dst, const uint8_t* src, uint64_t n, hipStream_t stream);

// Fused encode + per-shard HighwayHash (one pass).  p: the encode RowSet with
// in_off = data shards, out_off = parity shards, base == out_base; h: key and
// digest output [n][C+R][32].  C <= 16, R <= 4, any shard length.
bool fused_supported(int C, int R, uint64_t shard_len);
// RS(12,4): the fused encode as the one-pass network heal of every parity
// shard (rs_decode_netq.hip, k_encode_hash_net12); its 4 x 12 coefficient
// rows, which the launch's tables must match.
const uint8_t* encode_net12_coef();
hipError_t launch_encode_hash_net12(GfApplyParams p, HashParams h, uint64_t shard_len, uint64_t n_stripes,
                                    hipStream_t stream);
// ... and RS(10,4)'s (k_decode_records_net10 over rs104_decode_nets.h).
const uint8_t* encode_net10_coef();
hipError_t launch_encode_hash_net10(GfApplyParams p, HashParams h, uint64_t shard_len, uint64_t n_stripes,
                                    hipStream_t stream);
// The fused encode + HH256S on the run-time-table one-pass kernel for any k
// <= 16, m <= 4 (rs_decode.hip, ENC).
hipError_t launch_encode_hash_table(GfApplyParams p, HashParams h, uint64_t shard_len, uint64_t n_stripes,
                                    hipStream_t stream);
// ... and RS(8,4)'s, RS(6,4)'s (rs_decode_net.hip, 8-stripe
// workgroups, two network waves).
const uint8_t* encode_net_coef();
const uint8_t* encode_net6_coef();
hipError_t launch_encode_hash_net(GfApplyParams p, HashParams h, uint64_t shard_len, uint64_t n_stripes,
                                  hipStream_t stream);
hipError_t launch_encode_hash_net6(GfApplyParams p, HashParams h, uint64_t shard_len, uint64_t n_stripes,
                                   hipStream_t stream);
// One-pass degraded GET (k_decode_records_dma) for RS(k, m), k <= 16, m <= 4,
// any shard length (a ragged last step), over nf (k..k+m-1) present record
// files — and EC:5..8 (m <= k, k + m <= 16) with one or two files absent:
// false if the shape is not supported.
bool decode_dma_supported(int k, int m, int nf, uint64_t shard_len);
// coef: the launch's R x k coefficient rows (host memory, row-major), matched
// against the compile-time XOR-network patterns (rs_decode_net.hip); may be null.
// A listed pattern runs its network; otherwise the table kernel runs if
// `any_table` (a forced one-pass engine) or table_one_pass_preferred(k, R),
// else hipErrorNotSupported (the caller takes the two-pass path).
hipError_t launch_decode_records_dma(GfApplyParams p, HashParams h, int k, int m, int nf, uint64_t shard_len,
                                     uint64_t n_stripes, const uint8_t* coef, bool any_table, hipStream_t stream);
// One-pass heal (k_decode_records_dma with target hashing), the same
// geometries: nf present source files, `targets` absent target files written
// with digests (nf + targets <= k + m).  A pattern with a compile-time network
// runs it; otherwise the table kernel runs if `any_table` (a forced one-pass
// engine) or table_one_pass_preferred(k, R), else hipErrorNotSupported: the
// caller takes the two-pass path.
bool heal_dma_supported(int k, int m, int nf, int targets, uint64_t shard_len);
// The run-time-table one-pass kernel against the two-pass path for k
// survivors and R rows (rebuilt / healed + compared), two_per_cu: the launch
// shape fits two workgroups a CU (rs_decode.hip).
bool table_one_pass_preferred(int k, int R, bool two_per_cu);
// The fused encode + HH256S (config 4's kernel for other geometries) on the
// run-time-table one-pass kernel with ENC, where it measured faster than the
// packed k_encode_hash_fused at 1 MiB blocks, n = 4096 (k >= 9: 2-9 %,
// profiles/r05/fused_table/; k = 4..8 since round 6's gf_rows: 2-9 %, RS(3,3)
// 3 %, profiles/r06/fused_table/) — not RS(4,3) / RS(5,3) (1-5 % slower),
// RS(2,2) (13 % slower), RS(3,2) (level) or k + m > 16.
constexpr bool table_enc_geometry(int k, int m) {
    return m >= 1 && m <= 4 && k + m <= 16 && (k >= 4 || (k == 3 && m == 3)) && !(m == 3 && (k == 4 || k == 5));
}
hipError_t launch_heal_records_dma(GfApplyParams p, HashParams h, int k, int m, int nf, int targets,
                                   uint64_t shard_len, uint64_t n_stripes, const uint8_t* coef, bool any_table,
                                   hipStream_t stream);

// The one-pass GET/heal kernel with compile-time XOR networks
// (rs_decode_net.hip, k_decode_records_net): RS(8,4) patterns of one or two
// lost shards (rs84_decode_nets.h), built in RSG_NET_PARTS translation units.
#define RSG_NET_PARTS 8
// pattern id whose (heal, nf, R, n_store, R x 8 rows) equal the launch's, or -1
int records_net_pattern(int heal, int nf, int R, int n_store, const uint8_t* coef);
#define RSG_NET_PART_DECL(i)                                                                               \
    bool launch_records_net_part##i(int pid, uint64_t blocks, const GfApplyParams& p, const HashParams& h, \
                                    hipStream_t stream);
RSG_NET_PART_DECL(0)
RSG_NET_PART_DECL(1)
RSG_NET_PART_DECL(2)
RSG_NET_PART_DECL(3)
RSG_NET_PART_DECL(4)
RSG_NET_PART_DECL(5)
RSG_NET_PART_DECL(6)
RSG_NET_PART_DECL(7)
#undef RSG_NET_PART_DECL
// RS(10,4) (rs_decode_netq.hip built with RSG_NETQ_K=10, k_decode_records_net10): the same for R x 10 rows
int records_net10_pattern(int heal, int nf, int R, int n_store, const uint8_t* coef);
#define RSG_NET10_PART_DECL(i)                                                                                \
    bool launch_records_net10_part##i(int pid, uint64_t blocks, const GfApplyParams& p, const HashParams& h, \
                                      hipStream_t stream);
RSG_NET10_PART_DECL(0)
RSG_NET10_PART_DECL(1)
RSG_NET10_PART_DECL(2)
RSG_NET10_PART_DECL(3)
RSG_NET10_PART_DECL(4)
RSG_NET10_PART_DECL(5)
RSG_NET10_PART_DECL(6)
RSG_NET10_PART_DECL(7)
#undef RSG_NET10_PART_DECL
// RS(6,4) (rs_decode_net.hip built with RSG_NET_K=6, k_decode_records_net6): the same for R x 6 rows
int records_net6_pattern(int heal, int nf, int R, int n_store, const uint8_t* coef);
#define RSG_NET6_PART_DECL(i)                                                                                \
    bool launch_records_net6_part##i(int pid, uint64_t blocks, const GfApplyParams& p, const HashParams& h, \
                                     hipStream_t stream);
RSG_NET6_PART_DECL(0)
RSG_NET6_PART_DECL(1)
RSG_NET6_PART_DECL(2)
RSG_NET6_PART_DECL(3)
RSG_NET6_PART_DECL(4)
RSG_NET6_PART_DECL(5)
RSG_NET6_PART_DECL(6)
RSG_NET6_PART_DECL(7)
#undef RSG_NET6_PART_DECL
// RS(12,4) (rs_decode_netq.hip, k_decode_records_net12): the same for R x 12 rows
int records_net12_pattern(int heal, int nf, int R, int n_store, const uint8_t* coef);
#define RSG_NET12_PART_DECL(i)                                                                               \
    bool launch_records_net12_part##i(int pid, uint64_t blocks, const GfApplyParams& p, const HashParams& h, \
                                      hipStream_t stream);
RSG_NET12_PART_DECL(0)
RSG_NET12_PART_DECL(1)
RSG_NET12_PART_DECL(2)
RSG_NET12_PART_DECL(3)
RSG_NET12_PART_DECL(4)
RSG_NET12_PART_DECL(5)
RSG_NET12_PART_DECL(6)
RSG_NET12_PART_DECL(7)
#undef RSG_NET12_PART_DECL
// One-pass heal possible for this shape (the table kernel takes every k <=
// 16, m <= 4, and EC:5..8's heals of one or two targets; which kernel runs is
// decided at launch).
bool heal_one_pass_shape(int k, int m, int nf, int targets, uint64_t shard_len);
hipError_t launch_encode_hash_fused(GfApplyParams p, HashParams h, uint64_t shard_len, uint64_t n_stripes,
                                    hipStream_t stream);

// Ring variant (one stripe per workgroup, E encoder waves, E KiB chunks,
// double-buffered LDS rows) for batches of few large stripes.  Requires
// shard_len % (1024*E) == 0, E in {1,2,4}, C <= 16, R <= 4.
size_t ring_lds_bytes(int C, int R, uint32_t E);
bool ring_supported(int C, int R, uint64_t shard_len, uint32_t E);
hipError_t launch_encode_hash_ring(GfApplyParams p, HashParams h, uint64_t shard_len, uint64_t n_stripes,
                                   uint32_t E, hipStream_t stream);

}  // namespace rsg
