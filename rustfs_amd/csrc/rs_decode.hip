// rs_decode.hip — the one-pass GET / heal kernel with run-time coefficient
// tables (k_decode_records_dma) and its launchers.  Compiled once per survivor
// count C = 1..16 with RSG_DECODE_C=C (Makefile: that part instantiates the
// C-survivor kernels, every present-file count and heal target count, and
// exports launch_get_tab_C), and once without it (the dispatch below), so the
// instantiations build in parallel.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "rs_device.h"
#include "rs_records.h"

namespace rsg {

// ---------------------------------------------------------------------------
// One-pass degraded GET (rsg_decode_records_dev, a data disk lost) for
// RS(k, m) with k <= 16 and m <= 4 (and EC:5..8, below): every present record of G
// stripes is verified, the missing data shards rebuilt from the first C = k
// present (survivors), the present data shards copied through and the
// surplus parity compared with its re-derived value — reading each present
// record once.  The k_encode_hash_dma layout: NF present files, G/2 x NF
// LDS-DMA instructions per 512-byte step (one shard of stripes i and i+G/2
// each) into a 3-slot ring; ceil(G NF / 16) DMA/hash waves (8 instructions
// each, 16 verify streams straight out of the ring) and G table-GF waves,
// one per stripe (survivor rows from the ring: rebuilt rows stored to the
// output, surplus rows compared against their ring rows, survivor data
// copied to the output).  One barrier per step.  The host redoes the stripes
// whose verify flags differ from the assumed pattern.  At most m rows
// (missing data + surplus parity, or heal targets + surplus) are ever needed:
// RM = 4 table slots, 8 for m > 4.
//   p: tab[r][c] over the C survivors (present files 0..C-1 of the launch),
//      rows [0, n_store) rebuilt into out_base + s*out_stripe_stride +
//      out_off[r], rows [n_store, R) compared with present file 8 + (r -
//      n_store); copy_mask/copy_off: survivors copied to the output;
//      ok_flags[s] cleared on a compare mismatch; units = S / 512.
//   h: base[f] = body of record 0 of present file f, stripe_stride = record
//      pitch, flag_base[f][s] cleared on a digest mismatch, key, n.
// TH > 0 is the one-pass heal (rsg_heal_records_dev): the TH stored rows are
// target record bodies (out_stripe_stride = record pitch, no copy-through);
// the GF waves also write them into a double-buffered LDS row area, and
// ceil(8 TH / 16) target-hasher waves hash them one step behind and write
// each target record's digest header (BitrotWriter::write).
// Issue priority of the wave roles in the DMA kernels (GfApplyParams::
// wave_prio): kPrioHash raises the hash waves, kPrioGf the GF / encoder
// waves.  Default kPrioGf: the GF waves of the one-pass GET/heal run ahead
// of the latency-bound hash chains instead of queueing behind them (RS(8,4),
// n = 4096: GET 2 lost 2.44 -> 2.18 ms, heal 1.92 -> 1.69 ms;
// profiles/r02/ab_prio/).  Tuning::get_prio overrides it for A/B runs.
[[maybe_unused]] static uint32_t dma_prio() { return (uint32_t)tuning().get_prio; }

// RD: ring slots (RD - 1 steps of DMA in flight).  3 by default; 2 for the
// 4-stripe workgroups of C > 8 survivors where the workgroup then fits half a
// CU's LDS, so two share a CU (two hash chains and two GF waves per SIMD),
// as the RS(12,4) network kernels do.
template <int NF, int G, int TH = 0, int RD = dma::D>
struct GetShape : RecRing<NF, G, TH> {
    // a heal on a 2-slot ring whose last hash wave's idle quads cover the
    // target streams hashes its targets there (records_hash_target_wave, LAG
    // 1): one wave fewer
    static constexpr bool MERGE = RD == 2 && TH > 0 && 2 * (8 - RecRing<NF, G, TH>::LAST) >= G * TH;
    static constexpr int WAVES = RecRing<NF, G, TH>::HW + G + (MERGE ? 0 : RecRing<NF, G, TH>::TW);
    static constexpr uint32_t LDS = RD * RecRing<NF, G, TH>::DSLOT + (TH ? 2 * RecRing<NF, G, TH>::TSLOT : 16);
    // waves per SIMD the register budget must allow (two workgroups per CU on a 2-slot ring)
    static constexpr int WPE = RD == 2 ? (2 * WAVES + 3) / 4 : 1;
};

// One step's GF rows 0..ROWS-1 of a table-kernel GF wave: acc[r] = sum over
// survivors c of tab[c][r] * x[c] (8 bytes a lane), the (c, r) terms in
// c-major order in units of 4, unit u + 1's coefficient tables read from the
// LDS while unit u's perms run (sched_barrier keeps that order; 2 x 20
// registers of tables), one basic block a step.  Rows past ROWS are not
// touched.  (A loop with a per-row `r < R` exit made every term its own block
// with its LDS read's latency exposed: RS(8,8) GET 2.74 -> 2.35 ms, RS(9,4)
// 1.59 -> 1.52 this way; computing all RM rows whatever R instead cost more
// than that where R < RM: RS(3,2) GET, R = 2 of 4, 1.55 -> 1.78 ms;
// profiles/r06/gf_pipe/.)
template <int C, int RM, int ROWS>
__device__ __forceinline__ void gf_rows(const uint2 (&x)[C], const uint8_t* tb, uint32_t m7, uint32_t m3,
                                        uint32_t (&acc)[RM][2], uint32_t (&pend)[RM][2]) {
    constexpr int N = C * ROWS, UW = C > 8 ? 2 : 4, U = (N + UW - 1) / UW;  // (C > 8: 4 would spill)
    uint4 ta[2][UW];
    uint32_t tc[2][UW];
    auto load_unit = [&](int u, int b) {
#pragma unroll
        for (int j = 0; j < UW; ++j) {
            const int i = u * UW + j;
            if (i >= N) break;
            const uint8_t* tp = tb + ((i / ROWS) * RM + i % ROWS) * 32;
            ta[b][j] = *(const uint4*)tp;
            tc[b][j] = *(const uint32_t*)(tp + 16);
        }
    };
    load_unit(0, 0);
    // this variant's own masks: the selectors below are not hoisted above
    // the caller's choice of variant (all C x 6 live at once)
    asm volatile("" : "+v"(m7), "+v"(m3));
    uint32_t sel[C][6];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (u + 1 < U) load_unit(u + 1, (u + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < UW; ++j) {
            const int i = u * UW + j, c = i / ROWS, r = i % ROWS, b = u & 1;
            if (i >= N) break;
            if (r == 0) {
                sel[c][0] = x[c].x & m7, sel[c][1] = x[c].y & m7;
                sel[c][2] = (x[c].x >> 3) & m7, sel[c][3] = (x[c].y >> 3) & m7;
                sel[c][4] = (x[c].x >> 6) & m3, sel[c][5] = (x[c].y >> 6) & m3;
            }
            const uint4 t4 = ta[b][j];
            const uint32_t t2 = tc[b][j];
            gf_fold(c & 1, acc[r][0], pend[r][0], __builtin_amdgcn_perm(t4.y, t4.x, sel[c][0]),
                    __builtin_amdgcn_perm(t4.w, t4.z, sel[c][2]), __builtin_amdgcn_perm(t2, t2, sel[c][4]));
            gf_fold(c & 1, acc[r][1], pend[r][1], __builtin_amdgcn_perm(t4.y, t4.x, sel[c][1]),
                    __builtin_amdgcn_perm(t4.w, t4.z, sel[c][3]), __builtin_amdgcn_perm(t2, t2, sel[c][5]));
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

// gf_rows where a step has at least 16 (c, r) terms (fewer: the per-row loop
// is as fast — RS(3,2) GET, 6 terms, 1.60 against 1.66 ms); false otherwise.
template <int C, int RM, int ROWS>
__device__ __forceinline__ bool gf_rows_pipe(const uint2 (&x)[C], const uint8_t* tb, uint32_t m7, uint32_t m3,
                                             uint32_t (&acc)[RM][2], uint32_t (&pend)[RM][2]) {
    if constexpr (C * ROWS >= 16) {
        gf_rows<C, RM, ROWS>(x, tb, m7, m3, acc, pend);
        return true;
    } else {
        return false;
    }
}

// ENC: the fused encode + HH256S over a stripe buffer (launch_encode_hash_table:
// the heal of every parity shard, p.out_* the parity rows in place, every
// digest to h.out in the batch digest layout instead of verified / written
// record headers).
template <int C, int NF, int G, int TH, int RD = dma::D, int RM = 4, bool ENC = false>
__global__ __launch_bounds__((64 * GetShape<NF, G, TH, RD>::WAVES))
__attribute__((amdgpu_waves_per_eu(GetShape<NF, G, TH, RD>::WPE))) void k_decode_records_dma(const GfApplyParams p,
                                                                                            const HashParams h) {
    static_assert(C >= 1 && C <= kMaxC && (RM == 4 || RM == 8) && RM <= kMaxR && NF >= C && NF <= C + RM &&
                      TH <= RM && NF + TH <= C + RM,
                  "RS(C, <= RM)");
    using dma::CH;
    using dma::IP;
    using dma::PP;
    constexpr int D = RD;
    using L = GetShape<NF, G, TH, RD>;
    constexpr int SPW = L::SPW, HS = L::HS;
    __shared__ __attribute__((aligned(16))) uint8_t ring[D * L::DSLOT];
    __shared__ __attribute__((aligned(16))) uint8_t tabs[C * RM * 32];
    __shared__ __attribute__((aligned(16))) uint8_t trow[TH ? 2 * L::TSLOT : 16];
    static_assert(D * L::DSLOT + C * RM * 32 + (TH ? 2 * L::TSLOT : 16) <= 160 * 1024, "the ring fits the LDS");
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint64_t n = h.n;
    const uint32_t steps = p.units;
    const uint64_t s0 = (uint64_t)blockIdx.x * SPW;
    for (uint32_t i = threadIdx.x; i < (uint32_t)(C * RM); i += blockDim.x) {
        const int c = i / RM, r = i % RM;
        *(uint4*)(tabs + i * 32) = make_uint4(p.tab[r][c][0], p.tab[r][c][1], p.tab[r][c][2], p.tab[r][c][3]);
        *(uint32_t*)(tabs + i * 32 + 16) = p.tab[r][c][4];
    }
    // (the tables are published by B(0), which every wave passes before use)

    if constexpr (TH > 0 && !L::MERGE) {
        if (wave >= (uint32_t)(L::HW + SPW)) {
            records_target_hasher<G, TH, 1, ENC, 2, 0, false, L::WPE>(&karg_gf(), &karg_hash(), trow,
                                                                       wave - L::HW - SPW, steps, s0);
            return;
        }
    }
    if constexpr (L::MERGE) {
        if (wave == (uint32_t)(L::HW - 1)) {  // the last hash wave hashes the target rows too
            records_hash_target_wave<NF, G, RD, TH, 2, L::TSLOT, 1, false, L::WPE, ENC>(&karg_gf(), &karg_hash(), ring, trow, wave, steps, s0);
            return;
        }
    }
    if (wave >= (uint32_t)L::HW) {
        // ------------------------- GF wave: one stripe -------------------------
        if (p.wave_prio & kPrioGf) __builtin_amdgcn_s_setprio(2);
        const uint32_t e = wave - L::HW;
        const uint64_t stripe = s0 + e;
        const bool live = stripe < n;
        uint8_t* ob = p.out_base + (live ? stripe : 0) * p.out_stripe_stride + lane * 8u;
        const uint32_t R = p.R, nst = p.n_store, cmask = p.copy_mask;
        const uint32_t m7 = vgpr_const(0x07070707u), m3 = vgpr_const(0x03030303u);
        const uint32_t tail = walk_tail(p.byte_end, steps);  // a ragged walk's last step: first tail bytes only
        // row of present file f for this stripe: instruction f*HS + e%HS, half e/HS
        const uint32_t roff = (e % HS) * IP + (e / HS) * CH + lane * 8u;
        bool bad = false;  // this lane saw a surplus-parity mismatch
        lds_barrier();  // B(0)
#pragma unroll 1
        for (uint32_t s = 0; s < steps; ++s) {
            const uint8_t* slot = ring + (s % D) * L::DSLOT + roff;
            uint2 x[C];
#pragma unroll
            for (int c = 0; c < C; ++c) x[c] = *(const uint2*)(slot + c * HS * IP);
            uint32_t tz;  // opaque zero: table reads stay at their use
            asm volatile("s_mov_b32 %0, 0" : "=s"(tz));
            const uint8_t* tb = tabs + tz;
            uint32_t acc[RM][2], pend[RM][2];
#pragma unroll
            for (int r = 0; r < RM; ++r) acc[r][0] = acc[r][1] = pend[r][0] = pend[r][1] = 0u;
            // R rows a step, R = RM or (RM = 4) fewer: the rebuilt rows plus the
            // surplus compared, m rows for a data-shard loss (wave-uniform)
            bool piped = false;
            if constexpr (RM == 4) {
                if (R == 4) piped = gf_rows_pipe<C, 4, 4>(x, tb, m7, m3, acc, pend);
                else if (R == 3) piped = gf_rows_pipe<C, 4, 3>(x, tb, m7, m3, acc, pend);
                else if (R == 2) piped = gf_rows_pipe<C, 4, 2>(x, tb, m7, m3, acc, pend);
                else piped = gf_rows_pipe<C, 4, 1>(x, tb, m7, m3, acc, pend);
            } else {  // EC:5..8: m rows for a data-shard loss, m = 5..8
                if (R == 8) piped = gf_rows_pipe<C, RM, 8>(x, tb, m7, m3, acc, pend);
                else if (R == 7) piped = gf_rows_pipe<C, RM, 7>(x, tb, m7, m3, acc, pend);
                else if (R == 6) piped = gf_rows_pipe<C, RM, 6>(x, tb, m7, m3, acc, pend);
                else if (R == 5) piped = gf_rows_pipe<C, RM, 5>(x, tb, m7, m3, acc, pend);
            }
            if (!piped) {  // few terms, or EC:5..8 with at most 4 rows: per row
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    const uint32_t s0a = x[c].x & m7, s0b = x[c].y & m7;
                    const uint32_t s1a = (x[c].x >> 3) & m7, s1b = (x[c].y >> 3) & m7;
                    const uint32_t s2a = (x[c].x >> 6) & m3, s2b = (x[c].y >> 6) & m3;
#pragma unroll
                    for (int r = 0; r < RM; ++r) {
                        if ((uint32_t)r >= R) break;  // wave-uniform
                        const uint8_t* tp = tb + (c * RM + r) * 32;
                        const uint4 t4 = *(const uint4*)tp;
                        const uint32_t t2 = *(const uint32_t*)(tp + 16);
                        gf_fold(c & 1, acc[r][0], pend[r][0], __builtin_amdgcn_perm(t4.y, t4.x, s0a),
                                __builtin_amdgcn_perm(t4.w, t4.z, s1a), __builtin_amdgcn_perm(t2, t2, s2a));
                        gf_fold(c & 1, acc[r][1], pend[r][1], __builtin_amdgcn_perm(t4.y, t4.x, s0b),
                                __builtin_amdgcn_perm(t4.w, t4.z, s1b), __builtin_amdgcn_perm(t2, t2, s2b));
                    }
                }
            }
            if constexpr (C & 1) {  // an odd survivor count leaves its last coefficient's third term pending
#pragma unroll
                for (int r = 0; r < RM; ++r) {
                    acc[r][0] ^= pend[r][0];
                    acc[r][1] ^= pend[r][1];
                }
            }
            // the rows exist here, whatever uses them below (not sunk into the
            // conditional store / compare blocks, with their table reads)
#pragma unroll
            for (int r = 0; r < RM; ++r) asm volatile("" : "+v"(acc[r][0]), "+v"(acc[r][1]));
            const bool part = s + 1 == steps && tail != CH;  // wave-uniform
            const uint64_t keep = part ? part_mask8(lane * 8u, tail) : ~0ull;
#pragma unroll
            for (int r = 0; r < RM; ++r) {
                if ((uint32_t)r >= R) break;
                const uint2 v = make_uint2(acc[r][0], acc[r][1]);
                if ((uint32_t)r < nst) {
                    if (live) {
                        // cached 8-byte stores: the L2 gathers the rows' 512-byte
                        // steps (against non-temporal: GET -1 to -4 %, heal level,
                        // profiles/r05/ab_tc/)
                        if (!part) st64_any(ob + p.out_off[r] + (uint64_t)s * CH, u64_of(v));
                        else st64_part(ob + p.out_off[r] + (uint64_t)s * CH, u64_of(v), lane * 8u, tail);
                    }
                    if constexpr (TH > 0)
                        *(uint2*)(trow + (s & 1) * L::TSLOT + (r * SPW + e) * PP + lane * 8u) = v;
                } else {
                    const uint2 o = *(const uint2*)(slot + (C + (r - nst)) * HS * IP);
                    bad |= ((u64_of(o) ^ u64_of(v)) & keep) != 0ull;
                }
            }
            if (live) {
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    if (!((cmask >> c) & 1u)) continue;
                    if (!part) st16_nt_half(ob + p.copy_off[c] + (uint64_t)s * CH, x[c]);
                    else st64_part(ob + p.copy_off[c] + (uint64_t)s * CH, u64_of(x[c]), lane * 8u, tail);
                }
            }
            lds_barrier();  // B(s+1): done with slot s % D
        }
        // the stripe's surplus verdict, written whole (no memset before the launch)
        const bool any_bad = __builtin_amdgcn_ballot_w64(bad) != 0;
        if (live && nst < R && lane == 0) p.ok_flags[stripe] = any_bad ? 0 : 1;
        return;
    }
    // ------------------------- DMA + verify-hash wave -------------------------
    records_hash_wave<NF, G, 0, RD, ENC, L::WPE>(&karg_hash(), p.wave_prio, ring, wave, steps, s0);
}

// 4-stripe workgroups (C > 8) on a 2-slot ring where it fits half a CU's LDS
// and at most 8 waves (two workgroups: 4 a SIMD) — a heal's target hashing
// merged into its last hash wave where that wave has room.  9-wave shapes
// (RS(16,4) GET, RS(15,4) GET, RS(14,4) heal) fit two a CU at 96 registers
// too, but measured no better than on 3 slots, and slower than two passes
// (GET RS(16,4) 2.16 vs 1.78 ms, RS(15,4) 2.20 vs 2.10; profiles/r05/ab_rd2/)
template <int C, int NF, int G, int TH, int RM = 4>
constexpr int table_rd() {
    return (G == 4 && GetShape<NF, G, TH, 2>::LDS + C * RM * 32 <= 80 * 1024 - 512 &&
            GetShape<NF, G, TH, 2>::WAVES <= 8)
               ? 2
               : dma::D;
}

template <int C, int NF, int G, int TH = 0, int RM = 4, bool ENC = false>
static void launch_get(uint64_t blocks, const GfApplyParams& p, const HashParams& h, hipStream_t stream) {
    constexpr int RD = table_rd<C, NF, G, TH, RM>();
    hipLaunchKernelGGL((k_decode_records_dma<C, NF, G, TH, RD, RM, ENC>), dim3((uint32_t)blocks),
                       dim3(64 * GetShape<NF, G, TH, RD>::WAVES), 0, stream, p, h);
}

// nf present files -> the k_decode_records_dma<C, NF, G, TH> instantiation:
// kTabLaunched, kTabDeclined (not `any_table` and the two-pass path is the
// faster one, table_one_pass_preferred) or kTabInvalid
enum { kTabInvalid = 0, kTabLaunched = 1, kTabDeclined = 2 };
template <int C, int G, int TH, int NF>
static int launch_get_nf(int nf, uint64_t n_stripes, const GfApplyParams& p, const HashParams& h, bool any_table,
                         hipStream_t stream) {
    // (patterns of more than 16 shards are not built: rustfs stores at most
    // 16, MAX_ERASURE_SHARDS, fileinfo.rs:38 — one_pass_geometry)
    if constexpr (NF + (TH ? TH : 1) > C + 4 || NF + (TH ? TH : 1) > 16) {
        return kTabInvalid;
    } else {
        if (nf != NF) return launch_get_nf<C, G, TH, NF + 1>(nf, n_stripes, p, h, any_table, stream);
        if (!any_table && !table_one_pass_preferred(C, (int)p.R, table_rd<C, NF, G, TH>() == 2)) return kTabDeclined;
        const uint64_t blocks = (n_stripes + G - 1) / G;
        if (blocks > 0x7fffffffull) return kTabInvalid;
        launch_get<C, NF, G, TH>(blocks, p, h, stream);
        return kTabLaunched;
    }
}

using TabLaunch = int (*)(int nf, int th, uint64_t n_stripes, const GfApplyParams& p, const HashParams& h,
                          bool any_table, hipStream_t stream);

#define RSG_DEC_CAT2(a, b) a##b
#define RSG_DEC_CAT(a, b) RSG_DEC_CAT2(a, b)

using WideLaunch = int (*)(int m, int nf, int th, uint64_t n_stripes, const GfApplyParams& p, const HashParams& h,
                           bool any_table, hipStream_t stream);

#if defined(RSG_DECODE_C) && defined(RSG_DECODE_WIDE)
// Explicit storage classes EC:5..8 (m > 4 parity shards, m <= k, k + m <= 16
// drives: storageclass.rs:480-498, fileinfo.rs:38): the table kernel with up
// to RM = 8 rows (missing data + surplus parity, or heal targets + surplus)
// for every one- and two-loss pattern — GET with one or two files absent,
// heal of one target (the other files present, or one more absent) or two —
// and (round 6) GET with three to m files absent and the heal of all of
// them, in 4-stripe workgroups (the ring of up to 15 files would not fit 8).
// Other patterns (a heal of some of several lost shards) take the two-pass
// path.
// Preferred (not forced): as table_one_pass_preferred, and the heal of five
// or more lost shards (9-wave workgroups, one a CU: RS(8,8) heal of 5 lost
// 2.74 vs 3.21 ms two-pass, RS(10,6) of 6 2.23 vs 2.62), but not a GET that
// rebuilds 8 rows (RS(8,8) with every data shard lost: 2.70 vs 2.25 ms;
// profiles/r06/ec58/many_lost/).
template <int C, int NF, int TH>
static int launch_wide(uint64_t n_stripes, const GfApplyParams& p, const HashParams& h, bool any_table,
                       hipStream_t stream) {
    constexpr int G = 4, RM = 8;
    const bool pref = (TH >= 5 || table_one_pass_preferred(C, (int)p.R, table_rd<C, NF, G, TH, RM>() == 2)) &&
                      !(TH == 0 && p.n_store >= 8);
    if (!any_table && !pref) return kTabDeclined;
    const uint64_t blocks = (n_stripes + G - 1) / G;
    if (blocks > 0x7fffffffull) return kTabInvalid;
    launch_get<C, NF, G, TH, RM>(blocks, p, h, stream);
    return kTabLaunched;
}

// L = 5..M files lost: the GET (th = 0) and the heal of all L (th = L)
template <int C, int M, int L>
static int launch_wide_many(int nf, int th, uint64_t n_stripes, const GfApplyParams& p, const HashParams& h,
                            bool any_table, hipStream_t stream) {
    if constexpr (L > M) {
        return kTabInvalid;
    } else {
        constexpr int T = C + M;
        if (nf == T - L && th == 0) return launch_wide<C, T - L, 0>(n_stripes, p, h, any_table, stream);
        if (nf == T - L && th == L) return launch_wide<C, T - L, L>(n_stripes, p, h, any_table, stream);
        return launch_wide_many<C, M, L + 1>(nf, th, n_stripes, p, h, any_table, stream);
    }
}

template <int C, int M>
static int launch_wide_m(int nf, int th, uint64_t n_stripes, const GfApplyParams& p, const HashParams& h,
                         bool any_table, hipStream_t stream) {
    if constexpr (M > C || C + M > 16) {
        return kTabInvalid;
    } else {
        constexpr int T = C + M;
        if (th == 0 && nf == T - 1) return launch_wide<C, T - 1, 0>(n_stripes, p, h, any_table, stream);
        if (th == 0 && nf == T - 2) return launch_wide<C, T - 2, 0>(n_stripes, p, h, any_table, stream);
        if (th == 1 && nf == T - 1) return launch_wide<C, T - 1, 1>(n_stripes, p, h, any_table, stream);
        if (th == 1 && nf == T - 2) return launch_wide<C, T - 2, 1>(n_stripes, p, h, any_table, stream);
        if (th == 2 && nf == T - 2) return launch_wide<C, T - 2, 2>(n_stripes, p, h, any_table, stream);
        // three to m files lost (round 6): the GET, and the heal of every
        // lost shard — still at most m rows (missing + surplus)
        if (th == 0 && nf == T - 3) return launch_wide<C, T - 3, 0>(n_stripes, p, h, any_table, stream);
        if (th == 0 && nf == T - 4) return launch_wide<C, T - 4, 0>(n_stripes, p, h, any_table, stream);
        if (th == 3 && nf == T - 3) return launch_wide<C, T - 3, 3>(n_stripes, p, h, any_table, stream);
        if (th == 4 && nf == T - 4) return launch_wide<C, T - 4, 4>(n_stripes, p, h, any_table, stream);
        return launch_wide_many<C, M, 5>(nf, th, n_stripes, p, h, any_table, stream);
    }
}

int RSG_DEC_CAT(launch_get_wide_, RSG_DECODE_C)(int m, int nf, int th, uint64_t n_stripes, const GfApplyParams& p,
                                                const HashParams& h, bool any_table, hipStream_t stream) {
    constexpr int C = RSG_DECODE_C;
    switch (m) {
        case 5: return launch_wide_m<C, 5>(nf, th, n_stripes, p, h, any_table, stream);
        case 6: return launch_wide_m<C, 6>(nf, th, n_stripes, p, h, any_table, stream);
        case 7: return launch_wide_m<C, 7>(nf, th, n_stripes, p, h, any_table, stream);
        case 8: return launch_wide_m<C, 8>(nf, th, n_stripes, p, h, any_table, stream);
    }
    return kTabInvalid;
}
#elif defined(RSG_DECODE_C)
// This part's fused encode + HH256S (k = C data shards, m = 1..4 parity):
// the heal of every parity shard with ENC — built where the fused launcher
// takes it (table_enc_geometry, rs_kernels.h); false elsewhere.
template <int C, int M>
static bool launch_enc_m(uint64_t blocks, const GfApplyParams& p, const HashParams& h, hipStream_t stream) {
    if constexpr (!table_enc_geometry(C, M)) {
        return false;
    } else {
        launch_get<C, C, get_group(C), M, 4, true>(blocks, p, h, stream);
        return true;
    }
}
bool RSG_DEC_CAT(launch_enc_tab_, RSG_DECODE_C)(int m, uint64_t n_stripes, const GfApplyParams& p,
                                                const HashParams& h, hipStream_t stream) {
    constexpr int C = RSG_DECODE_C, G = get_group(C);
    const uint64_t blocks = (n_stripes + G - 1) / G;
    if (blocks > 0x7fffffffull) return false;
    switch (m) {
        case 1: return launch_enc_m<C, 1>(blocks, p, h, stream);
        case 2: return launch_enc_m<C, 2>(blocks, p, h, stream);
        case 3: return launch_enc_m<C, 3>(blocks, p, h, stream);
        case 4: return launch_enc_m<C, 4>(blocks, p, h, stream);
    }
    return false;
}

// This part's survivor count: GET (th = 0) and heal (th = 1..4 targets).
int RSG_DEC_CAT(launch_get_tab_, RSG_DECODE_C)(int nf, int th, uint64_t n_stripes, const GfApplyParams& p,
                                               const HashParams& h, bool any_table, hipStream_t stream) {
    constexpr int C = RSG_DECODE_C, G = get_group(C);
    switch (th) {
        case 0: return launch_get_nf<C, G, 0, C>(nf, n_stripes, p, h, any_table, stream);
        case 1: return launch_get_nf<C, G, 1, C>(nf, n_stripes, p, h, any_table, stream);
        case 2: return launch_get_nf<C, G, 2, C>(nf, n_stripes, p, h, any_table, stream);
        case 3: return launch_get_nf<C, G, 3, C>(nf, n_stripes, p, h, any_table, stream);
        case 4: return launch_get_nf<C, G, 4, C>(nf, n_stripes, p, h, any_table, stream);
    }
    return kTabInvalid;
}
#else
int launch_get_tab_1(int, int, uint64_t, const GfApplyParams&, const HashParams&, bool, hipStream_t);
int launch_get_tab_2(int, int, uint64_t, const GfApplyParams&, const HashParams&, bool, hipStream_t);
int launch_get_tab_3(int, int, uint64_t, const GfApplyParams&, const HashParams&, bool, hipStream_t);
int launch_get_tab_4(int, int, uint64_t, const GfApplyParams&, const HashParams&, bool, hipStream_t);
int launch_get_tab_5(int, int, uint64_t, const GfApplyParams&, const HashParams&, bool, hipStream_t);
int launch_get_tab_6(int, int, uint64_t, const GfApplyParams&, const HashParams&, bool, hipStream_t);
int launch_get_tab_7(int, int, uint64_t, const GfApplyParams&, const HashParams&, bool, hipStream_t);
int launch_get_tab_8(int, int, uint64_t, const GfApplyParams&, const HashParams&, bool, hipStream_t);
int launch_get_tab_9(int, int, uint64_t, const GfApplyParams&, const HashParams&, bool, hipStream_t);
int launch_get_tab_10(int, int, uint64_t, const GfApplyParams&, const HashParams&, bool, hipStream_t);
int launch_get_tab_11(int, int, uint64_t, const GfApplyParams&, const HashParams&, bool, hipStream_t);
int launch_get_tab_12(int, int, uint64_t, const GfApplyParams&, const HashParams&, bool, hipStream_t);
int launch_get_tab_13(int, int, uint64_t, const GfApplyParams&, const HashParams&, bool, hipStream_t);
int launch_get_tab_14(int, int, uint64_t, const GfApplyParams&, const HashParams&, bool, hipStream_t);
int launch_get_tab_15(int, int, uint64_t, const GfApplyParams&, const HashParams&, bool, hipStream_t);
int launch_get_tab_16(int, int, uint64_t, const GfApplyParams&, const HashParams&, bool, hipStream_t);
bool launch_enc_tab_1(int, uint64_t, const GfApplyParams&, const HashParams&, hipStream_t);
bool launch_enc_tab_2(int, uint64_t, const GfApplyParams&, const HashParams&, hipStream_t);
bool launch_enc_tab_3(int, uint64_t, const GfApplyParams&, const HashParams&, hipStream_t);
bool launch_enc_tab_4(int, uint64_t, const GfApplyParams&, const HashParams&, hipStream_t);
bool launch_enc_tab_5(int, uint64_t, const GfApplyParams&, const HashParams&, hipStream_t);
bool launch_enc_tab_6(int, uint64_t, const GfApplyParams&, const HashParams&, hipStream_t);
bool launch_enc_tab_7(int, uint64_t, const GfApplyParams&, const HashParams&, hipStream_t);
bool launch_enc_tab_8(int, uint64_t, const GfApplyParams&, const HashParams&, hipStream_t);
bool launch_enc_tab_9(int, uint64_t, const GfApplyParams&, const HashParams&, hipStream_t);
bool launch_enc_tab_10(int, uint64_t, const GfApplyParams&, const HashParams&, hipStream_t);
bool launch_enc_tab_11(int, uint64_t, const GfApplyParams&, const HashParams&, hipStream_t);
bool launch_enc_tab_12(int, uint64_t, const GfApplyParams&, const HashParams&, hipStream_t);
bool launch_enc_tab_13(int, uint64_t, const GfApplyParams&, const HashParams&, hipStream_t);
bool launch_enc_tab_14(int, uint64_t, const GfApplyParams&, const HashParams&, hipStream_t);
bool launch_enc_tab_15(int, uint64_t, const GfApplyParams&, const HashParams&, hipStream_t);
bool launch_enc_tab_16(int, uint64_t, const GfApplyParams&, const HashParams&, hipStream_t);
int launch_get_wide_5(int, int, int, uint64_t, const GfApplyParams&, const HashParams&, bool, hipStream_t);
int launch_get_wide_6(int, int, int, uint64_t, const GfApplyParams&, const HashParams&, bool, hipStream_t);
int launch_get_wide_7(int, int, int, uint64_t, const GfApplyParams&, const HashParams&, bool, hipStream_t);
int launch_get_wide_8(int, int, int, uint64_t, const GfApplyParams&, const HashParams&, bool, hipStream_t);
int launch_get_wide_9(int, int, int, uint64_t, const GfApplyParams&, const HashParams&, bool, hipStream_t);
int launch_get_wide_10(int, int, int, uint64_t, const GfApplyParams&, const HashParams&, bool, hipStream_t);
int launch_get_wide_11(int, int, int, uint64_t, const GfApplyParams&, const HashParams&, bool, hipStream_t);

static int launch_get_any(int k, int m, int nf, int th, uint64_t n_stripes, const GfApplyParams& p,
                          const HashParams& h, bool any_table, hipStream_t stream) {
    if (m > 4) {
        static const WideLaunch wide[7] = {launch_get_wide_5, launch_get_wide_6,  launch_get_wide_7, launch_get_wide_8,
                                           launch_get_wide_9, launch_get_wide_10, launch_get_wide_11};
        if (k < 5 || k > 11 || m > 8 || th < 0 || th > m) return kTabInvalid;
        return wide[k - 5](m, nf, th, n_stripes, p, h, any_table, stream);
    }
    static const TabLaunch parts[16] = {launch_get_tab_1,  launch_get_tab_2,  launch_get_tab_3,  launch_get_tab_4,
                                        launch_get_tab_5,  launch_get_tab_6,  launch_get_tab_7,  launch_get_tab_8,
                                        launch_get_tab_9,  launch_get_tab_10, launch_get_tab_11, launch_get_tab_12,
                                        launch_get_tab_13, launch_get_tab_14, launch_get_tab_15, launch_get_tab_16};
    if (k < 1 || k > 16 || th < 0 || th > 4) return kTabInvalid;
    return parts[k - 1](nf, th, n_stripes, p, h, any_table, stream);
}

// Geometries with a one-pass kernel: every k <= 16 with m <= 4 and k + m <=
// 16 — every set of 2 to 16 drives (disks_layout.rs:25, MAX_ERASURE_SHARDS =
// 16 in fileinfo.rs:38) at its default parity (storageclass.rs:24-31), the
// reduced-redundancy class's one parity shard (storageclass.rs:99, 326-331)
// and explicit EC:1..4 — any shard length (a ragged last step, rs_records.h
// walk_tail).  Larger sets (RS(16,4): 20 shards) take the two-pass path.
static bool walk_length_ok(uint64_t shard_len) {
    return shard_len >= 1 && (shard_len + dma::CH - 1) / dma::CH <= 0xffffffffull;
}
static bool one_pass_geometry(int k, int m, uint64_t shard_len) {
    return k >= 1 && k <= 16 && m >= 1 && m <= 4 && k + m <= 16 && walk_length_ok(shard_len);
}
// ... and the explicit classes EC:5..8 (m <= k, k + m <= 16 drives:
// storageclass.rs:480-498) for their one- and two-loss patterns
// (launch_get_wide_C above)
static bool wide_geometry(int k, int m, uint64_t shard_len) {
    return m >= 5 && m <= 8 && m <= k && k + m <= 16 && walk_length_ok(shard_len);
}
static int rows_max(int m) { return m > 4 ? 8 : 4; }

bool decode_dma_supported(int k, int m, int nf, uint64_t shard_len) {
    if (wide_geometry(k, m, shard_len)) return nf >= k && nf < k + m;
    return one_pass_geometry(k, m, shard_len) && nf >= k && nf < k + m;
}

bool heal_dma_supported(int k, int m, int nf, int targets, uint64_t shard_len) {
    if (wide_geometry(k, m, shard_len))
        return (targets == 1 && nf >= k + m - 2 && nf <= k + m - 1) || (targets >= 2 && targets <= m && nf == k + m - targets);
    return one_pass_geometry(k, m, shard_len) && nf >= k && targets >= 1 && nf + targets <= k + m;
}

// The table kernel against the two-pass path (GF pass over every column, then
// a verify launch): its GF waves, one per stripe, apply k survivors x R rows
// of v_perm tables per step, so past some k*R they set the pace — unless two
// workgroups share a CU (`two_per_cu`: the 2-slot ring, table_rd), which
// doubles the GF waves a SIMD interleaves.  At 1 MiB blocks, n = 4096: one
// workgroup a CU wins up to k*R = 40 (profiles/r05/geom/) — RS(9,4) with 2
// lost (R = 4: 36) GET 1.57 vs 2.16 ms, heal 1.61 vs 2.53; RS(15,1) (15) GET
// 0.96 vs 1.64 — and loses beyond: RS(16,4) (64, 9 waves: one a CU) GET 2.35 vs
// 1.82, heal 2.32 vs 1.96.  Two a CU win past it (profiles/r05/ab_rd2/):
// RS(11,4) (44) GET 1.50 vs 2.26 ms, RS(13,3) (39) GET 1.25 vs 1.86.
bool table_one_pass_preferred(int k, int R, bool two_per_cu) { return two_per_cu || k * R <= 40; }

// Patterns with a compile-time XOR network (RS(6,4), RS(8,4):
// rs_decode_net.hip; RS(10,4), RS(12,4): rs_decode_netq.hip): the launch's
// coefficient rows are matched byte for byte against the generated table; a
// listed pattern runs its network kernel, anything else the run-time-table
// kernel above (RS(4,4) too: its networks were 2-5 % faster than the table
// kernel, profiles/r05/netab/, and were dropped in round 6 for build time).
// Tuning::decode_net = false (RSG_DECODE_NET=0) keeps the table kernel for
// A/B runs.
static bool launch_net_if_listed(int heal, int k, int m, int nf, const uint8_t* coef, uint64_t n_stripes,
                                 const GfApplyParams& p, const HashParams& h, hipStream_t stream) {
    if (m != 4 || !coef || !tuning().decode_net || p.C != (uint32_t)k) return false;
    using Part = bool (*)(int, uint64_t, const GfApplyParams&, const HashParams&, hipStream_t);
    if (k == 12 || k == 10) {
        const int pid = k == 12 ? records_net12_pattern(heal, nf, (int)p.R, (int)p.n_store, coef)
                                : records_net10_pattern(heal, nf, (int)p.R, (int)p.n_store, coef);
        if (pid < 0) return false;
        const uint64_t blocks = (n_stripes + 3) / 4;
        if (blocks > 0x7fffffffull) return false;
        static const Part parts12[RSG_NET_PARTS] = {launch_records_net12_part0, launch_records_net12_part1,
                                                    launch_records_net12_part2, launch_records_net12_part3,
                                                    launch_records_net12_part4, launch_records_net12_part5,
                                                    launch_records_net12_part6, launch_records_net12_part7};
        static const Part parts10[RSG_NET_PARTS] = {launch_records_net10_part0, launch_records_net10_part1,
                                                    launch_records_net10_part2, launch_records_net10_part3,
                                                    launch_records_net10_part4, launch_records_net10_part5,
                                                    launch_records_net10_part6, launch_records_net10_part7};
        return (k == 12 ? parts12 : parts10)[pid % RSG_NET_PARTS](pid, blocks, p, h, stream);
    }
    if (k != 8 && k != 6) return false;
    const int pid = k == 8 ? records_net_pattern(heal, nf, (int)p.R, (int)p.n_store, coef)
                           : records_net6_pattern(heal, nf, (int)p.R, (int)p.n_store, coef);
    if (pid < 0) return false;
    GfApplyParams q = p;
    q.cached_stores = tuning().get_cached ? 1u : 0u;
    const uint64_t blocks = (n_stripes + 7) / 8;
    if (blocks > 0x7fffffffull) return false;
    static const Part parts[RSG_NET_PARTS] = {launch_records_net_part0, launch_records_net_part1,
                                              launch_records_net_part2, launch_records_net_part3,
                                              launch_records_net_part4, launch_records_net_part5,
                                              launch_records_net_part6, launch_records_net_part7};
    static const Part parts6[RSG_NET_PARTS] = {launch_records_net6_part0, launch_records_net6_part1,
                                               launch_records_net6_part2, launch_records_net6_part3,
                                               launch_records_net6_part4, launch_records_net6_part5,
                                               launch_records_net6_part6, launch_records_net6_part7};
    return (k == 8 ? parts : parts6)[pid % RSG_NET_PARTS](pid, blocks, q, h, stream);
}

// The record files' layout the DMA ring can walk: LDS-DMA takes sources at
// any alignment, so records of any pitch (RS(12,4): 87414 bytes) qualify;
// the per-lane DMA offsets are 32-bit (up to G/2 records on plus a body).
static bool dma_records_walkable(const HashParams& h) { return 5 * h.stripe_stride < (1ull << 32); }

bool heal_one_pass_shape(int k, int m, int nf, int targets, uint64_t shard_len) {
    return heal_dma_supported(k, m, nf, targets, shard_len);
}

// hipErrorNotSupported: no network for this pattern and the table heal is not
// wanted (neither forced nor preferred for k) — the caller takes the two-pass path.
hipError_t launch_heal_records_dma(GfApplyParams p, HashParams h, int k, int m, int nf, int targets,
                                   uint64_t shard_len, uint64_t n_stripes, const uint8_t* coef, bool any_table,
                                   hipStream_t stream) {
    p.wave_prio = dma_prio();
    if (!heal_one_pass_shape(k, m, nf, targets, shard_len) || (int)p.C != k || n_stripes == 0 ||
        p.R > (uint32_t)rows_max(m) ||
        p.n_store != (uint32_t)targets || p.copy_mask || !dma_records_walkable(h) ||
        p.out_stripe_stride != h.stripe_stride)
        return hipErrorInvalidValue;
    p.units = (uint32_t)((shard_len + dma::CH - 1) / dma::CH);
    p.byte_end = shard_len;
    h.n = n_stripes;
    if (launch_net_if_listed(1, k, m, nf, coef, n_stripes, p, h, stream)) return hipGetLastError();
    const int r = launch_get_any(k, m, nf, targets, n_stripes, p, h, any_table, stream);
    if (r == kTabDeclined) return hipErrorNotSupported;
    if (r != kTabLaunched) return hipErrorInvalidValue;
    return hipGetLastError();
}

// The fused encode + HH256S on the run-time-table one-pass kernel (the heal
// of every parity shard over a stripe buffer in place, ENC): k data shards
// (1..16), m = p.R parity (1..4).  p: the encode's table launch (base ==
// out_base, in_off the data rows, out_off the parity rows); h: key, out.
hipError_t launch_encode_hash_table(GfApplyParams p, HashParams h, uint64_t shard_len, uint64_t n_stripes,
                                    hipStream_t stream) {
    using EncLaunch = bool (*)(int, uint64_t, const GfApplyParams&, const HashParams&, hipStream_t);
    static const EncLaunch parts[16] = {launch_enc_tab_1,  launch_enc_tab_2,  launch_enc_tab_3,  launch_enc_tab_4,
                                        launch_enc_tab_5,  launch_enc_tab_6,  launch_enc_tab_7,  launch_enc_tab_8,
                                        launch_enc_tab_9,  launch_enc_tab_10, launch_enc_tab_11, launch_enc_tab_12,
                                        launch_enc_tab_13, launch_enc_tab_14, launch_enc_tab_15, launch_enc_tab_16};
    const int k = (int)p.C, m = (int)p.R;
    if (k < 1 || k > 16 || m < 1 || m > 4 || n_stripes == 0 || !walk_length_ok(shard_len) || p.base != p.out_base ||
        p.stripe_stride != p.out_stripe_stride || 5 * p.stripe_stride >= (1ull << 32))
        return hipErrorInvalidValue;
    p.n_store = (uint32_t)m;
    p.copy_mask = 0;
    p.mode = GF_MODE_STORE_COMPARE;
    p.wave_prio = dma_prio();
    p.units = (uint32_t)((shard_len + dma::CH - 1) / dma::CH);
    p.byte_end = shard_len;
    h.len = shard_len;
    h.n = n_stripes;
    h.shards = (uint64_t)(k + m);
    h.stripe_stride = p.stripe_stride;
    h.nbases = (uint32_t)k;
    for (int c = 0; c < k; ++c) h.base[c] = p.base + p.in_off[c];
    if (!parts[k - 1](m, n_stripes, p, h, stream)) return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t launch_decode_records_dma(GfApplyParams p, HashParams h, int k, int m, int nf, uint64_t shard_len,
                                     uint64_t n_stripes, const uint8_t* coef, bool any_table, hipStream_t stream) {
    p.wave_prio = dma_prio();
    if (!decode_dma_supported(k, m, nf, shard_len) || (int)p.C != k || n_stripes == 0 ||
        p.R > (uint32_t)rows_max(m) ||
        p.n_store > p.R || !dma_records_walkable(h))
        return hipErrorInvalidValue;
    p.units = (uint32_t)((shard_len + dma::CH - 1) / dma::CH);
    p.byte_end = shard_len;
    h.n = n_stripes;
    if (launch_net_if_listed(0, k, m, nf, coef, n_stripes, p, h, stream)) return hipGetLastError();
    const int r = launch_get_any(k, m, nf, 0, n_stripes, p, h, any_table, stream);
    if (r == kTabDeclined) return hipErrorNotSupported;
    if (r != kTabLaunched) return hipErrorInvalidValue;
    return hipGetLastError();
}
#endif  // RSG_DECODE_C

}  // namespace rsg
