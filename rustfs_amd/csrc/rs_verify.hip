// rs_verify.hip — verify-only walks of BitrotWriter record files at unaligned
// pitches (the in-place GET with every data file present, the whole-file
// bitrot_verify: rsgpu.cpp launch_verify_group / bitrot_verify_dev) through
// the record kernels' LDS-DMA ring instead of k_hh256_quad's per-lane 8-byte
// loads.  At 1 MiB blocks most geometries put their records off 8-byte
// alignment (RS(12,4): 32 + 87382 bytes, records at 6 mod 8), and the quad
// kernel's unaligned loads cost it ~7 % against the same walk at 0 mod 32
// (tools/verify_align_probe.py: 1.122 against 1.045 ms for 16 files x 4096
// records); global_load_lds takes the unaligned sources and lands them in LDS
// in order, where the hash waves read them aligned (rs_records.h
// records_hash_wave).  The workgroup is the record ring of 4 stripes (records
// r, r+1, r+2, r+3 of every file) and NF files with hash waves only.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <string.h>

#include "rs_device.h"
#include "rs_kernels.h"
#include "rs_records.h"

#ifndef RSG_VERIFY_DMA
#define RSG_VERIFY_DMA 1  // 0: never (A/B builds)
#endif

namespace rsg {

namespace {

constexpr int kVG = 4;  // records per file per workgroup

// Up to 12 files: a 3-slot ring (two steps of DMA in flight), two workgroups
// a CU; 13-15 files: a 2-slot ring (RS(10,4)'s 14 files 10 % faster than the
// quad kernel; RS(12,4)'s 16, 1 % slower, stay on it).  Launches of 13-15
// files at odd record pitches stay on the quad kernel's funnel (RS(14,2)'s 16:
// 12 % slower on the ring), more files too; split launches of 8 + 8 files
// measured 12-24 % slower than either, and 2-record workgroups on a 3-slot
// ring past 12 files 12-30 % slower (profiles/r05/ab_verify/, g2/).
template <int NF>
struct VerifyShape : RecRing<NF, kVG> {
    static constexpr int RD = NF <= 12 ? 3 : 2;
    static constexpr uint32_t LDS = RD * RecRing<NF, kVG>::DSLOT;
    static constexpr int PER_CU = (160 * 1024) / LDS > 8 ? 8 : (160 * 1024) / LDS;  // workgroups a CU holds
    static constexpr int WAVES = RecRing<NF, kVG>::HW;
    static constexpr int WPE = (PER_CU * WAVES + 3) / 4;
};

template <int NF>
__global__ __launch_bounds__(64 * VerifyShape<NF>::WAVES)
__attribute__((amdgpu_waves_per_eu(VerifyShape<NF>::WPE))) void k_verify_records_dma(const GfApplyParams p,
                                                                                     const HashParams h) {
    using L = VerifyShape<NF>;
    __shared__ __attribute__((aligned(16))) uint8_t ring[L::LDS];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t s0 = (uint64_t)blockIdx.x * kVG;
    (void)h;
    records_hash_wave<NF, kVG, 0, L::RD, false, L::WPE>(&karg_hash(), p.wave_prio, ring, wave, p.units, s0);
}

using VerifyLaunch = void (*)(uint64_t blocks, const GfApplyParams& p, const HashParams& h, hipStream_t stream);

template <int NF>
void launch_nf(uint64_t blocks, const GfApplyParams& p, const HashParams& h, hipStream_t stream) {
    static_assert(VerifyShape<NF>::LDS <= 160 * 1024, "the ring fits the LDS");
    hipLaunchKernelGGL((k_verify_records_dma<NF>), dim3((uint32_t)blocks), dim3(64 * VerifyShape<NF>::WAVES), 0,
                       stream, p, h);
}

constexpr int kMaxRingFiles = 15;
static_assert(VerifyShape<12>::LDS <= 80 * 1024 && VerifyShape<15>::LDS <= 80 * 1024, "two workgroups a CU");
const VerifyLaunch kLaunch[kMaxRingFiles + 1] = {
    nullptr,       launch_nf<1>,  launch_nf<2>,  launch_nf<3>,  launch_nf<4>,  launch_nf<5>,
    launch_nf<6>,  launch_nf<7>,  launch_nf<8>,  launch_nf<9>,  launch_nf<10>, launch_nf<11>,
    launch_nf<12>, launch_nf<13>, launch_nf<14>, launch_nf<15>};

}  // namespace

// A multi-file verify launch as launch_hh256 takes it (h.nbases files of
// h.per_base records at pitch h.stripe_stride, digest 32 bytes before each
// body, flags per file and record, no copies): run on the DMA ring when the
// records sit off 16-byte alignment (VerifyShape: which file counts and
// pitches).  false: not taken (the caller launches k_hh256_quad).
// The kernel writes each record's flag whole (1 verified, 0 not), where the
// quad kernel only clears.
bool launch_verify_records_dma(const HashParams& h, hipStream_t stream) {
    if (!RSG_VERIFY_DMA || h.nbases < 1 || h.nbases > (uint32_t)kMaxRingFiles || h.digest_off != -32 ||
        h.len == 0 || h.per_base == 0 || h.flags)
        return false;
    bool aligned = h.stripe_stride % 16 == 0;
    for (uint32_t b = 0; b < h.nbases; ++b) {
        if (h.copy_base[b] || !h.flag_base[b]) return false;
        aligned = aligned && (uintptr_t)h.base[b] % 16 == 0;
    }
    if (aligned) return false;  // the quad kernel's loads are aligned: nothing to gain
    bool odd = h.stripe_stride % 2 != 0;
    for (uint32_t b = 0; b < h.nbases; ++b) odd = odd || (uintptr_t)h.base[b] % 2 != 0;
    if (h.nbases > 12 && odd) return false;
    const uint64_t steps = (h.len + dma::CH - 1) / dma::CH;
    const uint64_t blocks = (h.per_base + kVG - 1) / kVG;
    // per-lane DMA offsets are 32-bit: HS records and a body
    if (steps > 0xffffffffull || blocks > 0x7fffffffull || 3 * h.stripe_stride >= (1ull << 32)) return false;
    GfApplyParams p;
    memset(&p, 0, sizeof(p));
    p.units = (uint32_t)steps;
    p.wave_prio = 0;
    HashParams q = h;
    q.n = h.per_base;  // the ring's stripes: the records of each file
    kLaunch[h.nbases](blocks, p, q, stream);
    return true;
}

}  // namespace rsg
