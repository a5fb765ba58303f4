// rs_records.h — the wave roles the one-pass GET / heal kernels share
// (rs_decode.hip k_decode_records_dma with run-time-table GF waves,
// rs_decode_net.hip k_decode_records_net with compile-time XOR-network
// waves): the LDS-DMA + verify-hash waves that bring every present record
// into the ring and check its digest (split_and_verify, bitrot.rs:227-247),
// and the target hashers of the heal (BitrotWriter::write, bitrot.rs:464-510).
// Internal; included once per translation unit after rs_device.h.
#pragma once

#include "rs_device.h"

namespace rsg {

// The record waves below are functions of their own (noinline): one copy per
// ring shape and role, called once per wave, instead of one inlined copy per
// pattern kernel — the per-pattern network kernels compile in half the time.
// They read the kernel's arguments where they lie, in the kernarg segment:
// every record kernel takes (const GfApplyParams p, const HashParams h), laid
// out in that order at their natural alignment.  (Taking the address of a
// by-value kernel argument instead makes the compiler copy it to scratch,
// ~1 KiB per lane.)
#define RSG_KARG const __attribute__((address_space(4)))
using KGf = RSG_KARG GfApplyParams;
using KHash = RSG_KARG HashParams;
__device__ __forceinline__ KGf& karg_gf() { return *(KGf*)__builtin_amdgcn_kernarg_segment_ptr(); }
__device__ __forceinline__ KHash& karg_hash() {
    constexpr size_t off = (sizeof(GfApplyParams) + alignof(HashParams) - 1) / alignof(HashParams) * alignof(HashParams);
    return *(KHash*)((RSG_KARG char*)__builtin_amdgcn_kernarg_segment_ptr() + off);
}
// OCC (template argument): the calling kernel's waves per SIMD
// (amdgpu_waves_per_eu) — a function shared by kernels of different
// occupancy gets the loosest register budget among them (RS(13,3)'s heal
// kernel took its target hasher's 129 registers, so one workgroup a CU);
// instantiating per occupancy keeps each at its kernels' budget.
#define RSG_RECORD_WAVE __device__ __attribute__((noinline))
// A called function takes its arguments in VGPRs: the wave-uniform ones are
// made scalar again on entry (SGPRs, SALU) as they were in the kernel.
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni(uint64_t v) {
    return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v);
}
template <class T>
__device__ __forceinline__ T* uni(T* v) {
    return (T*)(uintptr_t)uni((uint64_t)(uintptr_t)v);
}
__device__ __forceinline__ KGf& uni(KGf* v) { return *(KGf*)(uintptr_t)uni((uint64_t)(uintptr_t)v); }
__device__ __forceinline__ KHash& uni(KHash* v) { return *(KHash*)(uintptr_t)uni((uint64_t)(uintptr_t)v); }

// Ring of one workgroup: G stripes, NF present files, 512-byte steps.
// Present file f of stripe e sits in DMA instruction f*HS + e%HS, half e/HS
// (stripes e and e + HS share one 1 KiB LDS row pair of pitch IP).
template <int NF, int G, int TH = 0>
struct RecRing {
    static constexpr int SPW = G, HS = G / 2;                     // stripes per workgroup, per DMA half
    static constexpr int NI = HS * NF;                            // DMA instructions per step
    static constexpr uint32_t DSLOT = NI * dma::IP;
    static constexpr int HW = (NI + 7) / 8;                       // DMA/hash waves
    static constexpr int LAST = NI - 8 * (HW - 1);                // instructions of the last one
    static constexpr uint32_t TSLOT = SPW * (TH ? TH : 1) * dma::PP;  // one step of target rows
    static constexpr int TW = (SPW * TH + 15) / 16;               // target-hasher waves
};

// A record walk of shard_len S bytes takes steps = ceil(S / CH) steps of CH
// bytes; the last one holds `tail` = S - (steps - 1) CH bytes (1..CH).  A
// ragged walk (tail < CH: RS(12,4) at 1 MiB blocks has S = 87382, 170 whole
// steps and 342 bytes) brings its last step in through registers, byte-exact
// (nothing past a record body is read: the last record of a file may end the
// caller's buffer), hashes its whole packets and then HighwayHash's
// remainder packet; the GF waves store and compare only its first tail bytes.
__device__ __forceinline__ uint32_t walk_tail(uint64_t S, uint32_t steps) {
    return (uint32_t)(S - (uint64_t)(steps - 1) * dma::CH);
}

// The bytes of this lane's 8 at step offset `off` that lie before `valid`
// (all ones when the whole 8 do; the partial last step's compares).
__device__ __forceinline__ uint64_t part_mask8(uint32_t off, uint32_t valid) {
    if (off >= valid) return 0ull;
    if (off + 8 <= valid) return ~0ull;
    return (1ull << (8 * (valid - off))) - 1ull;
}

// DMA + verify-hash wave hw of a workgroup whose first stripe is s0: brings
// its (up to) 8 DMA instructions of every step into the RD-slot ring RD-1 steps ahead
// and hashes both halves of each straight out of the ring (quad j: instruction
// 8 hw + (j & 7), half j >> 3); at the end lane 0 of each live quad writes its
// record's verify flag whole (no memset before the launch).  One barrier per
// step: B(0) before step 0, B(s+1) after step s.  Record bodies may sit at any
// address (LDS-DMA takes unaligned sources); a ragged walk's last step is
// loaded by the same wave through registers (walk_tail).
// ENC (the fused encode + HH256S, k_encode_hash_net12): the sources are the
// data shards of a stripe buffer and each digest is written, not checked, to
// h.out + (stripe * h.shards + file) * 32 (the batch digest layout).
template <int NF, int G, int XB = 0, int RD = dma::D, bool ENC = false, int OCC = 0>
RSG_RECORD_WAVE void records_hash_wave(KHash* h_in, uint32_t wave_prio, uint8_t* ring_in, uint32_t hw_in,
                                       uint32_t steps_in, uint64_t s0_in) {
    KHash& h = uni(h_in);
    uint8_t* const ring = uni(ring_in);
    const uint32_t hw = uni(hw_in), steps = uni(steps_in);
    const uint64_t s0 = uni(s0_in);
    wave_prio = uni(wave_prio);
    using dma::CH;
    using dma::IP;
    constexpr int D = RD;  // ring slots: D - 1 steps of DMA in flight
    using dma::vmcnt_imm;
    using L = RecRing<NF, G>;
    constexpr int HS = L::HS;
    if (wave_prio & kPrioHash) __builtin_amdgcn_s_setprio(2);
    const uint32_t lane = threadIdx.x & 63u, q = lane & 3u, j = lane >> 2;
    const uint64_t n = h.n;
    const uint32_t ring_base = (uint32_t)(uintptr_t)ring;
    const int ndi = (hw == (uint32_t)(L::HW - 1)) ? L::LAST : 8;  // instructions this wave owns
    const uint32_t idx = 8 * hw + (j & 7u), half = j >> 3;
    const bool quad_on = (int)(j & 7u) < ndi;
    const uint32_t file = quad_on ? idx / HS : 0, stripe_l = (idx % HS) + HS * half;
    const uint32_t roff = (quad_on ? idx : 0) * IP + half * CH + 8 * q;
    const bool live = quad_on && s0 + stripe_l < n;
    const uint32_t tail = walk_tail(h.len, steps);
    const bool ragged = tail != CH;
    HHQuad st;
    {
        const uint64_t key[4] = {h.key[0], h.key[1], h.key[2], h.key[3]};
        hhq_init(st, key, q);
    }
    // record sources as a wave-uniform base (SGPRs) + a 32-bit per-lane
    // offset (the upper half's stripe, or the lower one again past n): the
    // loads take the saddr form, a step costs HS VALU adds
    uint64_t ubo[HS];
    uint32_t vlane[HS];
#pragma unroll
    for (int i = 0; i < HS; ++i) {
        const uint64_t lo = s0 + i, hi = lo + HS;
        ubo[i] = (lo < n ? lo : 0) * h.stripe_stride;
        vlane[i] = (lane & 31u) * 16u + ((lane >> 5) && hi < n ? (uint32_t)(HS * h.stripe_stride) : 0u);
    }
    // each instruction's record base, read from the kernel arguments once
    // (indexed by the wave's instructions, they were re-read every step)
    const uint8_t* ibase[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t ins = 8 * hw + (k < ndi ? k : 0);
        ibase[k] = h.base[ins / HS] + ubo[k % HS];
    }
    // the last step's hash: 16 packets from the ring (a ragged step: its
    // whole packets, then the remainder packet)
    auto hash_step = [&](uint32_t s) {
        uint64_t w[16];
        dma::read16(ring_base + (s % D) * L::DSLOT + roff, w);
        if (!ragged || s + 1 < steps) {
#pragma unroll
            for (int t = 0; t < 16; ++t) hhq_update(st, w[t]);
        } else {
            const uint32_t full = tail / 32;
#pragma unroll
            for (int t = 0; t < 16; ++t)
                if ((uint32_t)t < full) hhq_update(st, w[t]);  // wave-uniform
            if (tail % 32)
                hhq_remainder(st, (const uint8_t*)ring + (s % D) * L::DSLOT + roff - 8 * q + full * 32, tail % 32, q);
        }
    };
    // DMA of one step; false (nothing issued) for a ragged walk's last step
    auto dma_step = [&](uint32_t step) -> bool {
        if (ragged && step + 1 == steps) return false;
        uint32_t voff[HS];
#pragma unroll
        for (int i = 0; i < HS; ++i) voff[i] = vlane[i] + step * CH;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (k >= ndi) break;  // wave-uniform
            const uint32_t ins = 8 * hw + k;
            const uint8_t* src = ibase[k] + (uint64_t)voff[k % HS];
            __builtin_amdgcn_global_load_lds(
                (const void*)src, (__attribute__((address_space(3))) void*)(ring + (step % D) * L::DSLOT + ins * IP), 16,
                0, 0);
        }
        return true;
    };
    // the ragged last step through registers: 16 bytes per lane per
    // instruction, zero past the record body, then into its ring slot
    uint64_t tlo[8], thi[8];
    auto tail_load = [&]() {
        const uint32_t boff = (steps - 1) * CH + (lane & 31u) * 16u;  // offset in the record body
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (k >= ndi) break;
            const uint8_t* src = ibase[k] + (uint64_t)vlane[k % HS] + (steps - 1) * CH;
            tlo[k] = ld64_part(src, boff, h.len);
            thi[k] = ld64_part(src + 8, boff + 8, h.len);
        }
    };
    auto tail_store = [&]() {
        __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (k >= ndi) break;
            const uint32_t ins = 8 * hw + k;
            *(uint4*)(ring + ((steps - 1) % D) * L::DSLOT + ins * IP + lane * 16u) =
                make_uint4((uint32_t)tlo[k], (uint32_t)(tlo[k] >> 32), (uint32_t)thi[k], (uint32_t)(thi[k] >> 32));
        }
    };
    // the next step's DMA has landed (D - 2 steps younger in flight); after a
    // step with nothing issued, everything in flight
    auto wait_next = [&](bool issued) {
        if (!issued) __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
        else if (ndi == 8) __builtin_amdgcn_s_waitcnt(vmcnt_imm((D - 2) * 8));
        else __builtin_amdgcn_s_waitcnt(vmcnt_imm((D - 2) * L::LAST));
    };
    bool issued = true;
#pragma unroll
    for (int d = 0; d < D - 1; ++d) issued = dma_step(d < (int)steps ? d : steps - 1);
    if (ragged && steps == 1) {  // the only step is the ragged one
        tail_load();
        tail_store();
    }
    wait_next(issued);  // DMA(0) landed
    lds_barrier();  // B(0)
#pragma unroll 1
    for (uint32_t s = 0; s + 1 < steps; ++s) {
        issued = dma_step(s + D - 1 < steps ? s + D - 1 : steps - 1);  // into the slot step s-1 used
        const bool fill = ragged && s + 2 == steps;  // the ragged last step is next
        uint64_t w[16];
        dma::read16(ring_base + (s % D) * L::DSLOT + roff, w);
#pragma unroll
        for (int t = 0; t < 16; ++t) hhq_update(st, w[t]);
        if (fill) {  // after the packets: tlo/thi and w[] never live together (78-90 VGPRs, not 103)
            tail_load();
            tail_store();
        }
        wait_next(issued);
        lds_barrier();  // B(s+1)
    }
    {  // the last step (whole or ragged: its whole packets, then the remainder packet)
        const uint32_t s = steps - 1;
        if (!ragged) (void)dma_step(s);  // the clamped tail DMA (keeps every wave's count uniform)
        hash_step(s);
        wait_next(!ragged);
        lds_barrier();  // B(steps)
    }
    __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));  // the clamped tail DMA has landed before the wave ends
#pragma unroll
    for (int b = 0; b < XB; ++b) lds_barrier();  // B(steps+1 ..): roles that trail the DMA by XB more steps
    if constexpr (ENC) {  // the shard's digest (BitrotWriter's hash of the block it writes)
        if (live) hhq_finish(st, h.out + ((s0 + stripe_l) * h.shards + file) * 32, q);
        return;
    }
    // verify before use (split_and_verify, bitrot.rs:227-247): lane 0 of each
    // live quad writes its record's flag whole (no memset before the launch)
    const uint64_t d = hhq_digest(st, q);
    bool mis = false;
    if (live) mis = d != ld64_any(h.base[file] + (s0 + stripe_l) * h.stripe_stride - 32 + 8 * q);
    const uint64_t bal = __builtin_amdgcn_ballot_w64(mis);
    if (live && q == 0) h.flag_base[file][s0 + stripe_l] = ((bal >> lane) & 0xFull) ? 0 : 1;
}

// The last DMA + verify-hash wave of a heal workgroup whose idle quads
// (16 - 2 LAST of them: its instructions cover half the wave) take over the
// target hasher's streams (TTH target rows x G stripes), so the workgroup has
// one wave fewer — RS(12,4)'s heal of one data + one parity shard: 8 waves
// instead of 9, which is what lets two workgroups share a CU (5 waves on a
// SIMD left 96 registers a wave: 12 spilled).  Ring quads walk their records
// exactly as records_hash_wave (same DMA pipeline and barriers, XB = LAG - 1);
// target quad tq hashes target row stream tq (row tq / G of stripe tq % G) LAG
// steps behind the DMA from the target area (TNS slots of TSLOT bytes at
// `trow`, the rows at pitch PP) — ZERO: clearing what it read (the network
// kernels' accumulators; LAG 1: the table kernel's GF waves write whole rows) —
// and at the end writes the target record's digest header
// (BitrotWriter::write).  steps + LAG barriers.
template <int NF, int G, int RD, int TTH, int TNS, uint32_t TSLOT, int LAG = 2, bool ZERO = true, int OCC = 0,
          bool ENC = false>
RSG_RECORD_WAVE void records_hash_target_wave(KGf* p_in, KHash* h_in, uint8_t* ring_in, uint8_t* trow_in,
                                              uint32_t hw_in, uint32_t steps_in, uint64_t s0_in) {
    KGf& p = uni(p_in);
    KHash& h = uni(h_in);
    uint8_t* const ring = uni(ring_in);
    uint8_t* const trow = uni(trow_in);
    const uint32_t hw = uni(hw_in), steps = uni(steps_in);
    const uint64_t s0 = uni(s0_in);
    using dma::CH;
    using dma::IP;
    using dma::PP;
    constexpr int D = RD;
    using dma::vmcnt_imm;
    using L = RecRing<NF, G>;
    constexpr int HS = L::HS;
    constexpr int NDI = L::LAST;  // this (last) wave's instructions
    static_assert(2 * (8 - NDI) >= G * TTH && TTH > 0, "the idle quads cover the target streams");
    if (p.wave_prio & kPrioHash) __builtin_amdgcn_s_setprio(2);
    const uint32_t lane = threadIdx.x & 63u, q = lane & 3u, j = lane >> 2;
    const uint64_t n = h.n;
    const uint32_t ring_base = (uint32_t)(uintptr_t)ring, trow_base = (uint32_t)(uintptr_t)trow;
    const uint32_t idx = 8 * hw + (j & 7u), half = j >> 3;
    const bool quad_on = (int)(j & 7u) < NDI;  // a ring quad
    const uint32_t file = quad_on ? idx / HS : 0, stripe_l = (idx % HS) + HS * half;
    const uint32_t roff = (quad_on ? idx : 0) * IP + half * CH + 8 * q;
    const bool live = quad_on && s0 + stripe_l < n;
    // target quad tq: stream tq = row tq / G of stripe tq % G
    const uint32_t tq = quad_on ? 0u : ((j & 7u) - NDI) + half * (8 - NDI);
    const bool ton = !quad_on && tq < (uint32_t)(G * TTH);
    const uint32_t tr = ton ? tq / G : 0, te = tq % G;
    const bool tlive = ton && s0 + te < n;
    const uint32_t troff = (ton ? tq : 0) * PP + 8 * q;
    const uint32_t tail = walk_tail(h.len, steps);
    const bool ragged = tail != CH;
    HHQuad st;
    {
        const uint64_t key[4] = {h.key[0], h.key[1], h.key[2], h.key[3]};
        hhq_init(st, key, q);
    }
    uint64_t ubo[HS];
    uint32_t vlane[HS];
#pragma unroll
    for (int i = 0; i < HS; ++i) {
        const uint64_t lo = s0 + i, hi = lo + HS;
        ubo[i] = (lo < n ? lo : 0) * h.stripe_stride;
        vlane[i] = (lane & 31u) * 16u + ((lane >> 5) && hi < n ? (uint32_t)(HS * h.stripe_stride) : 0u);
    }
    const uint8_t* ibase[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t ins = 8 * hw + (k < NDI ? k : 0);
        ibase[k] = h.base[ins / HS] + ubo[k % HS];
    }
    auto dma_step = [&](uint32_t step) -> bool {
        if (ragged && step + 1 == steps) return false;
        uint32_t voff[HS];
#pragma unroll
        for (int i = 0; i < HS; ++i) voff[i] = vlane[i] + step * CH;
#pragma unroll
        for (int k = 0; k < NDI; ++k) {
            const uint32_t ins = 8 * hw + k;
            const uint8_t* src = ibase[k] + (uint64_t)voff[k % HS];
            __builtin_amdgcn_global_load_lds(
                (const void*)src, (__attribute__((address_space(3))) void*)(ring + (step % D) * L::DSLOT + ins * IP), 16,
                0, 0);
        }
        return true;
    };
    uint64_t tlo[8], thi[8];
    auto tail_load = [&]() {
        const uint32_t boff = (steps - 1) * CH + (lane & 31u) * 16u;
#pragma unroll
        for (int k = 0; k < NDI; ++k) {
            const uint8_t* src = ibase[k] + (uint64_t)vlane[k % HS] + (steps - 1) * CH;
            tlo[k] = ld64_part(src, boff, h.len);
            thi[k] = ld64_part(src + 8, boff + 8, h.len);
        }
    };
    auto tail_store = [&]() {
        __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
#pragma unroll
        for (int k = 0; k < NDI; ++k) {
            const uint32_t ins = 8 * hw + k;
            *(uint4*)(ring + ((steps - 1) % D) * L::DSLOT + ins * IP + lane * 16u) =
                make_uint4((uint32_t)tlo[k], (uint32_t)(tlo[k] >> 32), (uint32_t)thi[k], (uint32_t)(thi[k] >> 32));
        }
    };
    auto wait_next = [&](bool issued) {
        if (!issued) __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
        else __builtin_amdgcn_s_waitcnt(vmcnt_imm((D - 2) * NDI));
    };
    // interval i (after B(i)): ring quads absorb ring step i (i < steps), target
    // quads target step i - LAG (LAG <= i < steps + LAG); `rag`: this quad's
    // step is the walk's ragged last one (its whole packets, then the remainder
    // packet)
    auto absorb = [&](uint32_t i) {
        const bool t_act = ton && i >= (uint32_t)LAG;
        const bool act = quad_on ? i < steps : t_act;
        const uint32_t ts = i - (uint32_t)LAG;
        const uint32_t a = quad_on ? ring_base + (i % D) * L::DSLOT + roff : trow_base + (ts % TNS) * TSLOT + troff;
        const bool rag = ragged && (quad_on ? i + 1 == steps : ts + 1 == steps);
        uint64_t w[16];
        dma::read16(a, w);
        if (act) {
            const uint32_t full = rag ? tail / 32 : 16u;
#pragma unroll
            for (int t = 0; t < 16; ++t)
                if ((uint32_t)t < full) hhq_update(st, w[t]);
            if (rag && tail % 32) {
                const uint8_t* tb = quad_on ? (const uint8_t*)ring + (i % D) * L::DSLOT + roff
                                            : (const uint8_t*)trow + (ts % TNS) * TSLOT + troff;
                hhq_remainder(st, tb - 8 * q + full * 32, tail % 32, q);
            }
        }
        if constexpr (ZERO) {
            if (t_act) dma::zero16(a);
        }
    };
    bool issued = true;
#pragma unroll
    for (int d = 0; d < D - 1; ++d) issued = dma_step(d < (int)steps ? d : steps - 1);
    if (ragged && steps == 1) {
        tail_load();
        tail_store();
    }
    wait_next(issued);
    lds_barrier();  // B(0)
#pragma unroll 1
    for (uint32_t s = 0; s + 1 < steps; ++s) {
        issued = dma_step(s + D - 1 < steps ? s + D - 1 : steps - 1);
        const bool fill = ragged && s + 2 == steps;
        absorb(s);
        if (fill) {
            tail_load();
            tail_store();
        }
        wait_next(issued);
        lds_barrier();  // B(s+1)
    }
    {  // the ring's last step
        const uint32_t s = steps - 1;
        if (!ragged) (void)dma_step(s);
        absorb(s);
        wait_next(!ragged);
        lds_barrier();  // B(steps)
    }
    __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
#pragma unroll
    for (int l = 0; l < LAG; ++l) {  // target steps steps - LAG .. steps - 1
        if (l > 0) lds_barrier();  // B(steps+l): the last target rows published
        absorb(steps + l);
    }
    // ring quads: verify before use (bitrot.rs:227-247); target quads: the
    // target record's digest header (BitrotWriter::write).  ENC (the fused
    // encode): every digest to the batch digest layout, data then parity.
    const uint64_t d = hhq_digest(st, q);
    if constexpr (ENC) {
        if (live) st64_any(h.out + ((s0 + stripe_l) * h.shards + file) * 32 + 8 * q, d);
        if (tlive) st64_any(h.out + ((s0 + te) * h.shards + p.C + tr) * 32 + 8 * q, d);
        return;
    }
    bool mis = false;
    if (live) mis = d != ld64_any(h.base[file] + (s0 + stripe_l) * h.stripe_stride - 32 + 8 * q);
    const uint64_t bal = __builtin_amdgcn_ballot_w64(mis);
    if (live && q == 0) h.flag_base[file][s0 + stripe_l] = ((bal >> lane) & 0xFull) ? 0 : 1;
    if (tlive) st64_any(p.out_base + (s0 + te) * p.out_stripe_stride + p.out_off[tr] - 32 + 8 * q, d);
}

// Target-hasher wave tw of a heal workgroup: quad j hashes target row stream
// pi = 16 tw + j (row r = pi / SPW of stripe pi % SPW) from the double-
// buffered LDS row area LAG steps behind the DMA (step t-LAG's rows,
// published by B(t); LAG = 1: the GF waves write a step's rows in the
// interval its data is in the ring), and writes the target record's digest
// header in front of its body at out_base + stripe * out_stripe_stride +
// out_off[r] - 32 (ENC: parity row r's digest to the batch digest layout, as
// shard p.C + r).  steps + LAG barriers.  The row area has NS slots of SLOT
// bytes (0: RecRing's TSLOT) used round robin; ZERO: each row cleared once
// hashed (k_decode_records_net12's fused encode keeps its rows in the
// network waves' accumulators).
template <int G, int TH, int LAG = 1, bool ENC = false, int NS = 2, uint32_t SLOT = 0, bool ZERO = false, int OCC = 0>
RSG_RECORD_WAVE void records_target_hasher(KGf* p_in, KHash* h_in, const uint8_t* trow_in, uint32_t tw_in,
                                           uint32_t steps_in, uint64_t s0_in) {
    KGf& p = uni(p_in);
    KHash& h = uni(h_in);
    const uint8_t* const trow = uni(trow_in);
    const uint32_t tw = uni(tw_in), steps = uni(steps_in);
    const uint64_t s0 = uni(s0_in);
    constexpr int SPW = G;
    constexpr uint32_t TSLOT = SLOT ? SLOT : RecRing<1, G, TH>::TSLOT;
    if (p.wave_prio & kPrioHash) __builtin_amdgcn_s_setprio(2);
    const uint32_t lane = threadIdx.x & 63u, q = lane & 3u;
    const uint32_t pi = 16 * tw + (lane >> 2);  // r * SPW + stripe
    const bool on = pi < (uint32_t)(SPW * TH);
    const uint32_t r = on ? pi / SPW : 0, e = pi % SPW;
    const bool live = on && s0 + e < h.n;
    const uint32_t roff = (on ? pi : 0) * dma::PP + 8 * q;
    const uint32_t tail = walk_tail(h.len, steps);
    HHQuad st;
    {
        const uint64_t key[4] = {h.key[0], h.key[1], h.key[2], h.key[3]};
        hhq_init(st, key, q);
    }
    lds_barrier();  // B(0)
#pragma unroll 1
    for (uint32_t t = 0; t < steps + LAG; ++t) {
        if (t >= (uint32_t)LAG) {  // target rows of step t-LAG, published by B(t)
            const uint32_t base = (uint32_t)(uintptr_t)trow + ((t - LAG) % NS) * TSLOT + roff;
            uint64_t w[16];
            dma::read16(base, w);
            if (t - LAG + 1 < steps || tail == dma::CH) {
#pragma unroll
                for (int i = 0; i < 16; ++i) hhq_update(st, w[i]);
            } else {  // the ragged last step: whole packets, then the remainder packet
                const uint32_t full = tail / 32;
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    if ((uint32_t)i < full) hhq_update(st, w[i]);  // wave-uniform
                if (tail % 32)
                    hhq_remainder(st, trow + ((t - LAG) % NS) * TSLOT + roff - 8 * q + full * 32, tail % 32, q);
            }
            if constexpr (ZERO) {
                if (on) dma::zero16(base);
            }
        }
        if (t + 1 < steps + LAG) lds_barrier();  // B(t+1)
    }
    if (!live) return;
    if constexpr (ENC) hhq_finish(st, h.out + ((s0 + e) * h.shards + p.C + r) * 32, q);
    else hhq_finish(st, p.out_base + (s0 + e) * p.out_stripe_stride + p.out_off[r] - 32, q);
}

// Stripes per workgroup of the one-pass GET/heal kernels for C survivors: 8
// (one workgroup of 13 waves per CU at RS(8,4)) while the ring of 3 x G/2 x
// NF KiB-rows fits the LDS, 4 for C = 16 (RS(16,4): up to 19 present files).
// (Four stripes per workgroup at RS(8,4) — two workgroups of 7 waves per CU —
// measured no faster, profiles/r02/ab_eng/.)
// (Four-stripe workgroups for C <= 8 too — two or three a CU — measured
// 2-110 % slower again in round 5: RS(5,4) GET 1.81 -> 2.58 ms, RS(4,4) heal
// 1.85 -> 2.97; profiles/r05/ab_group/.)
constexpr int get_group(int C) { return C > 8 ? 4 : 8; }

}  // namespace rsg
