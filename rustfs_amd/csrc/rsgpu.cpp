// rsgpu.cpp — host side of the MI355X erasure engine behind include/rsgpu.h.
//
// Owns: GF(2^8) host arithmetic for matrix construction and inversion (the
// part of reed_solomon_erasure::ReedSolomon::new / get_data_decode_matrix that
// stays on the host), per-(k,m) codec cache (erasure.rs:448-470
// cached_modern_reed_solomon, <= 64 entries) with a per-codec cache of decode
// plans keyed by the erasure pattern (the LRU the fork keeps for inverted
// matrices), per-device contexts, and the launch planning that maps every
// encode / reconstruct / verify onto one GPU primitive: out = M * in.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <list>
#include <map>
#include <memory>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rsgpu.h"
#include "rs_kernels.h"

namespace rsg {  // the kernel-choice knobs (rs_kernels.hip): 0 = ok, 1 = unknown name / bad value
int set_tuning(const char* name, const char* value);
int get_tuning(const char* name, char* out, size_t cap);
}  // namespace rsg

namespace {

// --------------------------------------------------------------------------
// GF(2^8) / 0x11D, generator 2 (docs/architecture/erasure-coding.md:41-50).

struct Gf {
    uint8_t exp[512];
    uint8_t log[256];
    Gf() {
        unsigned x = 1;
        for (int i = 0; i < 255; ++i) {
            exp[i] = (uint8_t)x;
            log[x] = (uint8_t)i;
            x <<= 1;
            if (x & 0x100) x ^= 0x11D;
        }
        for (int i = 255; i < 512; ++i) exp[i] = exp[i - 255];
        log[0] = 0;
    }
    uint8_t mul(uint8_t a, uint8_t b) const { return (a && b) ? exp[log[a] + log[b]] : 0; }
    uint8_t div(uint8_t a, uint8_t b) const {
        if (!a) return 0;
        int l = (int)log[a] - (int)log[b];
        return exp[l < 0 ? l + 255 : l];
    }
    uint8_t pow(uint8_t a, int n) const {
        if (n == 0) return 1;
        if (a == 0) return 0;
        return exp[((int)log[a] * n) % 255];
    }
};

const Gf& gf() {
    static const Gf g;
    return g;
}

using Mat = std::vector<uint8_t>;  // row-major

bool invert(int n, Mat& a) {
    const Gf& g = gf();
    Mat w((size_t)n * 2 * n, 0);
    for (int r = 0; r < n; ++r) {
        std::memcpy(&w[(size_t)r * 2 * n], &a[(size_t)r * n], n);
        w[(size_t)r * 2 * n + n + r] = 1;
    }
    for (int c = 0; c < n; ++c) {
        int p = c;
        while (p < n && w[(size_t)p * 2 * n + c] == 0) ++p;
        if (p == n) return false;
        if (p != c)
            for (int j = 0; j < 2 * n; ++j) std::swap(w[(size_t)p * 2 * n + j], w[(size_t)c * 2 * n + j]);
        uint8_t* row = &w[(size_t)c * 2 * n];
        const uint8_t piv = row[c];
        if (piv != 1)
            for (int j = 0; j < 2 * n; ++j) row[j] = g.div(row[j], piv);
        for (int r = 0; r < n; ++r) {
            if (r == c) continue;
            uint8_t* o = &w[(size_t)r * 2 * n];
            const uint8_t f = o[c];
            if (!f) continue;
            for (int j = 0; j < 2 * n; ++j) o[j] ^= g.mul(f, row[j]);
        }
    }
    for (int r = 0; r < n; ++r) std::memcpy(&a[(size_t)r * n], &w[(size_t)r * 2 * n + n], n);
    return true;
}

// vandermonde(k+m, k) * inv(top k x k)
bool build_matrix(int k, int m, Mat& out) {
    const Gf& g = gf();
    const int t = k + m;
    Mat v((size_t)t * k);
    for (int r = 0; r < t; ++r)
        for (int c = 0; c < k; ++c) v[(size_t)r * k + c] = g.pow((uint8_t)r, c);
    Mat top(v.begin(), v.begin() + (size_t)k * k);
    if (!invert(k, top)) return false;
    out.assign((size_t)t * k, 0);
    for (int r = 0; r < t; ++r)
        for (int c = 0; c < k; ++c) {
            uint8_t acc = 0;
            for (int i = 0; i < k; ++i) acc ^= g.mul(v[(size_t)r * k + i], top[(size_t)i * k + c]);
            out[(size_t)r * k + c] = acc;
        }
    return true;
}

// v_perm_b32 tables of coefficient c: T0 lo/hi, T1 lo/hi, T2 of the 3/3/2-bit
// split (rs_kernels.hip header).
void coef_tables(uint8_t c, uint32_t t[5]) {
    const Gf& g = gf();
    auto pack = [&](int shift, int first) {
        uint32_t v = 0;
        for (int i = 0; i < 4; ++i) v |= (uint32_t)g.mul(c, (uint8_t)((first + i) << shift)) << (8 * i);
        return v;
    };
    t[0] = pack(0, 0);
    t[1] = pack(0, 4);
    t[2] = pack(3, 0);
    t[3] = pack(3, 4);
    t[4] = pack(6, 0);
}

// --------------------------------------------------------------------------
// Codec cache.

struct DecodePlan {
    std::vector<int> survivors;  // first k present shards, ascending
    std::vector<int> missing;    // missing shard indices, ascending
    Mat inv;                     // k x k inverse of the survivor sub-matrix
};

struct Codec {
    int k, m;
    Mat matrix;  // (k+m) x k
    std::mutex mu;
    std::list<std::pair<std::string, std::shared_ptr<DecodePlan>>> lru;
    std::map<std::string, decltype(lru)::iterator> index;
    static constexpr size_t kMaxPlans = 254;

    std::shared_ptr<DecodePlan> plan(const uint8_t* present) {
        std::string key((size_t)(k + m), '\0');
        for (int i = 0; i < k + m; ++i) key[i] = present[i] ? 1 : 0;
        std::lock_guard<std::mutex> g(mu);
        auto it = index.find(key);
        if (it != index.end()) {
            lru.splice(lru.begin(), lru, it->second);
            return it->second->second;
        }
        auto p = std::make_shared<DecodePlan>();
        for (int i = 0; i < k + m; ++i) {
            if (present[i]) {
                if ((int)p->survivors.size() < k) p->survivors.push_back(i);
            } else {
                p->missing.push_back(i);
            }
        }
        if ((int)p->survivors.size() < k) return nullptr;
        p->inv.assign((size_t)k * k, 0);
        for (int s = 0; s < k; ++s)
            std::memcpy(&p->inv[(size_t)s * k], &matrix[(size_t)p->survivors[s] * k], k);
        if (!invert(k, p->inv)) return nullptr;
        lru.emplace_front(key, p);
        index[key] = lru.begin();
        if (lru.size() > kMaxPlans) {
            index.erase(lru.back().first);
            lru.pop_back();
        }
        return p;
    }
};

std::mutex g_codec_mu;
std::map<std::pair<int, int>, std::shared_ptr<Codec>> g_codecs;
constexpr size_t kMaxCodecs = 64;  // MODERN_REED_SOLOMON_CACHE_MAX_ENTRIES, erasure.rs:73

int check_geometry(int k, int m) {
    if (k <= 0) return RSG_ERR_ZERO_DATA_SHARDS;
    if (m < 0) return RSG_ERR_INVALID_ARG;
    if (k + m > RSG_MAX_TOTAL_SHARDS) return RSG_ERR_TOO_MANY_SHARDS;
    return RSG_OK;
}

std::shared_ptr<Codec> get_codec(int k, int m) {
    std::lock_guard<std::mutex> g(g_codec_mu);
    auto it = g_codecs.find({k, m});
    if (it != g_codecs.end()) return it->second;
    auto c = std::make_shared<Codec>();
    c->k = k;
    c->m = m;
    if (!build_matrix(k, m, c->matrix)) return nullptr;
    if (g_codecs.size() < kMaxCodecs) g_codecs[{k, m}] = c;
    return c;
}

// Row r of out = rows[r] . in  (R x C coefficient matrix).
struct RowSet {
    int R = 0, C = 0;
    Mat coef;                    // R x C
    std::vector<uint64_t> in_off, out_off;
    // copy-through (optional, C entries): input c is also stored verbatim at
    // output offset copy_off[c] when copy[c] != 0 (done by the first row group)
    std::vector<uint8_t> copy;
    std::vector<uint64_t> copy_off;
};

// Parity rows of the encode matrix over the data shards.
RowSet encode_rows(const Codec& cd, uint64_t pitch) {
    RowSet rs;
    rs.R = cd.m;
    rs.C = cd.k;
    rs.coef.assign(cd.matrix.begin() + (size_t)cd.k * cd.k, cd.matrix.end());
    for (int c = 0; c < cd.k; ++c) rs.in_off.push_back((uint64_t)c * pitch);
    for (int r = 0; r < cd.m; ++r) rs.out_off.push_back((uint64_t)(cd.k + r) * pitch);
    return rs;
}

// Rows producing shard `idx` from the survivors: inv[idx] for data shards,
// G[idx] * inv for parity shards (identical bytes to re-encoding from the
// rebuilt data, because inv maps each present data shard to itself).
void plan_row(const Codec& cd, const DecodePlan& p, int idx, uint8_t* row) {
    const int k = cd.k;
    if (idx < k) {
        std::memcpy(row, &p.inv[(size_t)idx * k], k);
        return;
    }
    const Gf& g = gf();
    for (int c = 0; c < k; ++c) {
        uint8_t acc = 0;
        for (int i = 0; i < k; ++i) acc ^= g.mul(cd.matrix[(size_t)idx * k + i], p.inv[(size_t)i * k + c]);
        row[c] = acc;
    }
}

bool is_survivor(const DecodePlan& p, int idx) {
    return std::find(p.survivors.begin(), p.survivors.end(), idx) != p.survivors.end();
}

// Shards a reconstruct in `mode` writes.  RSG_RECONSTRUCT_REENCODE_PARITY
// re-encodes every parity shard (erasure.rs:425-428, 505-561), but a parity
// shard that is one of the survivors re-encodes to itself byte for byte
// (G[p] * inv is the unit row selecting it, whatever the other shards hold),
// so it is not a target: no launch ever overwrites a shard another launch of
// the same product still reads (chained C > 16 inputs, R > 8 rows).
std::vector<int> reconstruct_targets(const Codec& cd, const DecodePlan& p, const uint8_t* present, int mode) {
    std::vector<int> targets;
    for (int i = 0; i < cd.k + cd.m; ++i) {
        const bool is_data = i < cd.k;
        if (is_data && !present[i]) targets.push_back(i);
        else if (!is_data && mode == RSG_RECONSTRUCT_MISSING && !present[i]) targets.push_back(i);
        else if (!is_data && mode == RSG_RECONSTRUCT_REENCODE_PARITY && !is_survivor(p, i)) targets.push_back(i);
    }
    return targets;
}

RowSet reconstruct_rows(const Codec& cd, const DecodePlan& p, const uint8_t* present, int mode, uint64_t pitch) {
    RowSet rs;
    rs.C = cd.k;
    for (int s : p.survivors) rs.in_off.push_back((uint64_t)s * pitch);
    const std::vector<int> targets = reconstruct_targets(cd, p, present, mode);
    rs.R = (int)targets.size();
    rs.coef.assign((size_t)rs.R * cd.k, 0);
    for (int r = 0; r < rs.R; ++r) {
        plan_row(cd, p, targets[r], &rs.coef[(size_t)r * cd.k]);
        rs.out_off.push_back((uint64_t)targets[r] * pitch);
    }
    return rs;
}

// --------------------------------------------------------------------------
// GPU dispatch of out = M * in over n stripes.

uint64_t round_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

int hip_status(hipError_t e) {
    if (e == hipSuccess) return RSG_OK;
    if (e == hipErrorOutOfMemory) return RSG_ERR_OUT_OF_MEMORY;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return RSG_ERR_NO_DEVICE;
    return RSG_ERR_DEVICE;
}


// Kernel parameter block for rows [r0, r0+4) x inputs [c0, c0+16) of rs.
void fill_params(const RowSet& rs, int r0, int c0, const uint8_t* base, uint8_t* out_base, uint64_t stride,
                 uint64_t out_stride, uint32_t mode, uint8_t* ok_flags, rsg::GfApplyParams& p) {
    const int R = std::min(rsg::kMaxR, rs.R - r0);
    const int C = std::min(rsg::kMaxC, rs.C - c0);
    std::memset(&p, 0, sizeof(p));
    p.base = base;
    p.out_base = out_base;
    p.stripe_stride = stride;
    p.out_stripe_stride = out_stride;
    for (int c = 0; c < C; ++c) p.in_off[c] = rs.in_off[c0 + c];
    for (int r = 0; r < R; ++r) p.out_off[r] = rs.out_off[r0 + r];
    for (int r = 0; r < R; ++r)
        for (int c = 0; c < C; ++c) coef_tables(rs.coef[(size_t)(r0 + r) * rs.C + c0 + c], p.tab[r][c]);
    p.ok_flags = ok_flags;
    p.C = (uint32_t)C;
    p.R = (uint32_t)R;
    p.mode = mode;
    if (r0 == 0 && !rs.copy.empty())
        for (int c = 0; c < C; ++c)
            if (rs.copy[c0 + c]) {
                p.copy_mask |= 1u << c;
                p.copy_off[c] = rs.copy_off[c0 + c];
            }
}

// Tuning::fused = false (RSG_FUSED=0) disables the fused encode+hash kernel
// (A/B measurements).
bool fused_enabled() { return rsg::tuning().fused; }

int apply_rows(const RowSet& rs, const uint8_t* base, uint8_t* out_base, uint64_t stride, uint64_t out_stride,
               uint64_t len, uint64_t n, uint32_t mode, uint8_t* ok_flags, hipStream_t stream);

// Compare mode over more than kMaxC inputs (k > 16: RS(20,4), RS(192,64), ...).
// A chained product (STORE, then XOR launches) cannot compare inside the
// chain, so the rows are computed into stream-ordered scratch (groups of
// stripes, <= ~256 MiB) and compared against their targets with identity rows
// (<= kMaxR per launch).  Same verdict as the one-pass compare: ok_flags[s]
// cleared where any row differs (erasure.rs:430-441).
int apply_rows_compare_wide(const RowSet& rs, const uint8_t* base, uint8_t* out_base, uint64_t stride,
                            uint64_t out_stride, uint64_t len, uint64_t n, uint8_t* ok_flags, hipStream_t stream) {
    const uint64_t pitch = round_up(len, 256);
    const uint64_t per_stripe = pitch * (uint64_t)rs.R;
    const uint64_t group = std::max<uint64_t>(1, std::min<uint64_t>(n, (256ull << 20) / per_stripe));
    uint8_t* tmp = nullptr;
    int st = hip_status(hipMallocAsync((void**)&tmp, (size_t)(group * per_stripe), stream));
    if (st) return st;
    RowSet enc = rs;
    for (int r = 0; r < rs.R; ++r) enc.out_off[r] = (uint64_t)r * pitch;
    for (uint64_t s0 = 0; s0 < n && !st; s0 += group) {
        const uint64_t cnt = std::min(group, n - s0);
        st = apply_rows(enc, base + s0 * stride, tmp, stride, per_stripe, len, cnt, rsg::GF_MODE_STORE, nullptr,
                        stream);
        for (int r0 = 0; r0 < rs.R && !st; r0 += rsg::kMaxR) {
            RowSet id;
            id.R = id.C = std::min(rsg::kMaxR, rs.R - r0);
            id.coef.assign((size_t)id.R * id.C, 0);
            for (int i = 0; i < id.R; ++i) {
                id.coef[(size_t)i * id.C + i] = 1;
                id.in_off.push_back((uint64_t)(r0 + i) * pitch);
                id.out_off.push_back(rs.out_off[r0 + i]);
            }
            st = apply_rows(id, tmp, out_base + s0 * out_stride, per_stripe, out_stride, len, cnt,
                            rsg::GF_MODE_COMPARE, ok_flags + s0, stream);
        }
    }
    const int fst = hip_status(hipFreeAsync(tmp, stream));
    return st ? st : fst;
}

int apply_rows(const RowSet& rs, const uint8_t* base, uint8_t* out_base, uint64_t stride, uint64_t out_stride,
               uint64_t len, uint64_t n, uint32_t mode, uint8_t* ok_flags, hipStream_t stream) {
    if (rs.R == 0 || n == 0 || len == 0) return RSG_OK;
    if (mode == rsg::GF_MODE_COMPARE && rs.C > rsg::kMaxC)
        return apply_rows_compare_wide(rs, base, out_base, stride, out_stride, len, n, ok_flags, stream);
    // The vector kernel's 16-byte accesses need no alignment (ld16/st16 in
    // rs_kernels.hip); only the len % 16 tail of each shard takes the byte path.
    const uint64_t units = len / 16;
    if (units > 0xffffffffull) return RSG_ERR_UNSUPPORTED;

    for (int r0 = 0; r0 < rs.R; r0 += rsg::kMaxR) {
        for (int c0 = 0; c0 < rs.C; c0 += rsg::kMaxC) {
            rsg::GfApplyParams p;
            fill_params(rs, r0, c0, base, out_base, stride, out_stride,
                        mode == rsg::GF_MODE_COMPARE ? mode : (c0 == 0 ? rsg::GF_MODE_STORE : rsg::GF_MODE_XOR),
                        ok_flags, p);
            if (units) {
                p.units = (uint32_t)units;
                int st = hip_status(rsg::launch_gf_apply_vec(p, n, stream));
                if (st) return st;
            }
            if (units * 16 < len) {
                p.byte_begin = units * 16;
                p.byte_end = len;
                int st = hip_status(rsg::launch_gf_apply_byte(p, n, stream));
                if (st) return st;
            }
        }
    }
    return RSG_OK;
}

// One pass that stores rows [0, n_store) (at out_base, out_stride) and compares
// rows [n_store, R) (at out_base + out_off, cmp_stride per stripe) into
// ok_flags: the GET rebuild and its surplus-parity check read the survivors
// once.  Needs R <= kMaxR and C <= kMaxC (callers fall back otherwise).
int apply_store_compare(const RowSet& rs, int n_store, const uint8_t* base, uint8_t* out_base, uint64_t stride,
                        uint64_t out_stride, uint64_t cmp_stride, uint64_t len, uint64_t n, uint8_t* ok_flags,
                        hipStream_t stream) {
    if (rs.R > rsg::kMaxR || rs.C > rsg::kMaxC) return RSG_ERR_UNSUPPORTED;
    if (rs.R == 0 || n == 0 || len == 0) return RSG_OK;
    const uint64_t units = len / 16;
    if (units > 0xffffffffull) return RSG_ERR_UNSUPPORTED;
    rsg::GfApplyParams p;
    fill_params(rs, 0, 0, base, out_base, stride, out_stride, rsg::GF_MODE_STORE_COMPARE, ok_flags, p);
    p.n_store = (uint32_t)n_store;
    p.cmp_stripe_stride = cmp_stride;
    int st;
    if (units) {
        p.units = (uint32_t)units;
        if ((st = hip_status(rsg::launch_gf_apply_vec(p, n, stream)))) return st;
    }
    if (units * 16 < len) {
        p.byte_begin = units * 16;
        p.byte_end = len;
        if ((st = hip_status(rsg::launch_gf_apply_byte(p, n, stream)))) return st;
    }
    return RSG_OK;
}

const uint64_t kMagicKey[4] = {0xcd8a238efa34e74bull, 0x528596bbe6833e26ull, 0x14449fa35d930f04ull,
                               0xa036de22139de097ull};
const uint64_t kLegacyKey[4] = {3, 4, 2, 1};

const uint64_t* hash_key(int algo) {
    if (algo == RSG_HASH_HIGHWAY256S) return kMagicKey;
    if (algo == RSG_HASH_HIGHWAY256S_LEGACY) return kLegacyKey;
    return nullptr;
}

int hash_messages(int algo, const uint8_t* d_data, uint64_t len, uint64_t n, uint64_t shards, uint64_t pitch,
                  uint64_t stride, uint8_t* d_out, hipStream_t stream) {
    const uint64_t* key = hash_key(algo);
    if (!key) return RSG_ERR_INVALID_ARG;
    rsg::HashParams h;
    std::memset(&h, 0, sizeof(h));
    h.data = d_data;
    h.len = len;
    h.n = n;
    h.shards = shards;
    h.shard_pitch = pitch;
    h.stripe_stride = stride;
    std::memcpy(h.key, key, sizeof(h.key));
    h.out = d_out;
    return hip_status(rsg::launch_hh256(h, stream));
}


}  // namespace

// --------------------------------------------------------------------------
// Context.

// One lane of the host-buffer API (rsg_encode / rsg_reconstruct / rsg_verify /
// rsg_hash): its own stream and device buffer, so calls from several host
// threads (the reference encodes from many tokio workers, encode.rs:511-526)
// run their copies and kernels concurrently instead of queueing on one lock.
struct HostLane {
    std::mutex mu;
    hipStream_t stream = nullptr;
    uint8_t* d_buf = nullptr;
    size_t cap = 0;

    int ensure(size_t bytes) {
        if (!stream) {
            hipError_t e = hipStreamCreateWithFlags(&stream, hipStreamNonBlocking);
            if (e != hipSuccess) return hip_status(e);
        }
        if (bytes <= cap) return RSG_OK;
        if (d_buf) (void)hipFree(d_buf);
        d_buf = nullptr;
        cap = 0;
        const size_t want = std::max(bytes, (size_t)1 << 20);
        hipError_t e = hipMalloc((void**)&d_buf, want);
        if (e != hipSuccess) return hip_status(e);
        cap = want;
        return RSG_OK;
    }
};

constexpr int kHostLanes = 8;

// Scratch of one record-engine call (GET / heal / bitrot_verify): the device
// verify flags and surplus verdicts, their page-locked mirror (the verdict
// D2H is a few tens of KB, where a pageable copy's staging costs more than
// the copy) and the timing marks of rsg_set_kernel_timing.  Calls take one
// from the context's pool, so concurrent calls never share scratch.
struct RecScratch {
    uint8_t* d = nullptr;
    size_t dcap = 0;
    uint8_t* h = nullptr;
    uint8_t* hdev = nullptr;  // h as the device addresses it
    size_t hcap = 0;
    bool timing = false;
    std::vector<hipEvent_t> tev;
    size_t tev_used = 0;

    RecScratch() = default;
    RecScratch(const RecScratch&) = delete;
    RecScratch& operator=(const RecScratch&) = delete;
    ~RecScratch() {  // the context's device is current (rsg_destroy / job release)
        if (d) (void)hipFree(d);
        if (h) (void)hipHostFree(h);
        for (hipEvent_t e : tev) (void)hipEventDestroy(e);
    }
    int ensure(size_t dbytes, size_t hbytes) {
        if (dbytes > dcap) {
            if (d) (void)hipFree(d);
            d = nullptr;
            dcap = 0;
            const size_t want = std::max(dbytes, (size_t)64 << 10);
            hipError_t e = hipMalloc((void**)&d, want);
            if (e != hipSuccess) return hip_status(e);
            dcap = want;
        }
        if (hbytes > hcap) {
            if (h) (void)hipHostFree(h);
            h = nullptr;
            hcap = 0;
            const size_t want = std::max(hbytes, (size_t)64 << 10);
            hipError_t e = hipHostMalloc((void**)&h, want, hipHostMallocDefault);
            if (e != hipSuccess) return hip_status(e);
            hcap = want;
            if ((e = hipHostGetDevicePointer((void**)&hdev, h, 0)) != hipSuccess) {
                (void)hipHostFree(h);
                h = hdev = nullptr;
                hcap = 0;
                return hip_status(e);
            }
        }
        return RSG_OK;
    }
    // the call's verdicts (bytes at src, written by its work on s) into h, by
    // a kernel on s (rsg::launch_copy_to_host)
    int copy_back(hipStream_t s, const uint8_t* src, size_t bytes) {
        return hip_status(rsg::launch_copy_to_host(hdev, src, bytes, s));
    }
    // HIP event pairs around the kernel launches on the call's stream
    void tmark(hipStream_t s) {
        if (!timing) return;
        if (tev_used == tev.size()) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return;
            tev.push_back(e);
        }
        (void)hipEventRecord(tev[tev_used++], s);
    }
    void tunmark() {  // drop the last mark (a launch that did not happen)
        if (timing && tev_used) --tev_used;
    }
    // summed kernel time once the stream has passed the last mark, or -1
    float tsum() {
        float sum = 0.f;
        for (size_t i = 0; i + 1 < tev_used; i += 2) {
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, tev[i], tev[i + 1]) == hipSuccess) sum += ms;
        }
        const float r = (timing && tev_used >= 2) ? sum : -1.f;
        tev_used = 0;
        return r;
    }
};

struct rsg_ctx {
    int device = 0;
    hipStream_t stream = nullptr;

    // record-engine scratch pool (RecScratch): taken per call, returned when
    // the call's ticket finishes
    std::mutex rec_mu;
    std::vector<std::unique_ptr<RecScratch>> rec_free;
    std::atomic<bool> timing{false};          // rsg_set_kernel_timing
    std::atomic<int> record_engine{RSG_RECORD_ENGINE_AUTO};  // rsg_set_record_engine
    std::atomic<float> last_kernel_ms{-1.f};  // the last finished timed record call
    std::atomic<int> fail_subbatch{-1};       // rsg_test_fail_subbatch: fault injection, tests only

    std::unique_ptr<RecScratch> take_scratch() {
        std::unique_ptr<RecScratch> sc;
        {
            std::lock_guard<std::mutex> g(rec_mu);
            if (!rec_free.empty()) {
                sc = std::move(rec_free.back());
                rec_free.pop_back();
            }
        }
        if (!sc) sc.reset(new RecScratch());
        sc->timing = timing.load();
        sc->tev_used = 0;
        return sc;
    }
    void give_scratch(std::unique_ptr<RecScratch> sc) {
        if (!sc) return;
        std::lock_guard<std::mutex> g(rec_mu);
        if (rec_free.size() < 16) rec_free.push_back(std::move(sc));  // else freed here
    }

    HostLane lanes[kHostLanes];
    std::atomic<unsigned> next_lane{0};

    // host-batch pipeline (rsg_encode_batch_host_submit): kPipeSlots
    // stream/staging pairs used round-robin by consecutive sub-batches of all
    // submitted jobs, so a slot's staging buffer is reused only after its own
    // stream has finished the previous sub-batch (stream order); a job's ticket
    // maps to one event per slot it used.
    static constexpr int kPipeSlots = 3;
    std::mutex pipe_mu;
    hipStream_t pipe_stream[kPipeSlots] = {};
    uint8_t* d_stage[kPipeSlots] = {};
    size_t stage_cap = 0;
    unsigned next_slot = 0;
    uint64_t next_ticket = 1;
    // A job's completion events, destroyed with the last reference: a ticket
    // waited on by several threads keeps its events alive until every waiter
    // has returned.  Record-engine jobs (GET / heal) also carry a host
    // finishing step, run once by the first waiter or poller that sees the
    // events complete (it reads the verdicts the job copied back and redoes
    // the rare stripes whose verified pattern differs from the assumed one);
    // every waiter gets its result.  The step's argument is the events'
    // status: a failed job only releases its scratch.
    struct Job {
        std::vector<hipEvent_t> done;
        std::function<int(int)> finish;
        std::mutex fin_mu;
        bool finished = false;
        int result = RSG_OK;
        Job() = default;
        Job(const Job&) = delete;
        Job& operator=(const Job&) = delete;
        ~Job() {
            for (hipEvent_t e : done) (void)hipEventDestroy(e);
        }
    };
    std::map<uint64_t, std::shared_ptr<Job>> jobs;

    // pipe_mu held.  Growing the staging buffers waits for every sub-batch in
    // flight (they may still be reading the old ones).
    int ensure_pipeline(size_t bytes) {
        for (int i = 0; i < kPipeSlots; ++i)
            if (!pipe_stream[i]) {
                hipError_t e = hipStreamCreateWithFlags(&pipe_stream[i], hipStreamNonBlocking);
                if (e != hipSuccess) return hip_status(e);
            }
        if (bytes <= stage_cap) return RSG_OK;
        for (int i = 0; i < kPipeSlots; ++i) {
            hipError_t e = hipStreamSynchronize(pipe_stream[i]);
            if (e != hipSuccess) return hip_status(e);
        }
        for (int i = 0; i < kPipeSlots; ++i) {
            if (d_stage[i]) (void)hipFree(d_stage[i]);
            d_stage[i] = nullptr;
        }
        stage_cap = 0;
        for (int i = 0; i < kPipeSlots; ++i) {
            hipError_t e = hipMalloc((void**)&d_stage[i], bytes);
            if (e != hipSuccess) return hip_status(e);
        }
        stage_cap = bytes;
        return RSG_OK;
    }
};

namespace {
int enter(rsg_ctx* ctx) {
    if (!ctx) return RSG_ERR_INVALID_ARG;
    return hip_status(hipSetDevice(ctx->device));
}
// A free host lane, locked: try every lane once starting round-robin, then
// wait on the starting one.
std::unique_lock<std::mutex> acquire_lane(rsg_ctx* ctx, HostLane*& lane) {
    const unsigned start = ctx->next_lane.fetch_add(1, std::memory_order_relaxed);
    for (int i = 0; i < kHostLanes; ++i) {
        HostLane& l = ctx->lanes[(start + i) % kHostLanes];
        std::unique_lock<std::mutex> g(l.mu, std::try_to_lock);
        if (g.owns_lock()) {
            lane = &l;
            return g;
        }
    }
    lane = &ctx->lanes[start % kHostLanes];
    return std::unique_lock<std::mutex>(lane->mu);
}

// Shards laid out back to back (the reference's encode_buffer block:
// [shard 0 .. shard k+m-1], S bytes each, erasure.rs:848-887) move with one
// copy per direction instead of one per shard.
bool contiguous(const uint8_t* const* shards, int first, int count, size_t len) {
    for (int i = 1; i < count; ++i)
        if (shards[first + i] != shards[first] + (size_t)i * len) return false;
    return true;
}

// The device's view of page-locked host memory it can address (hipHostMalloc'd
// or registered), or nullptr (pageable memory, another device's allocation).
// Both ends of [p, p + len) must resolve to the same allocation.
uint8_t* pinned_view(const uint8_t* p, size_t len, int device) {
    hipPointerAttribute_t a, b;
    if (hipPointerGetAttributes(&a, p) != hipSuccess || hipPointerGetAttributes(&b, p + len - 1) != hipSuccess) {
        (void)hipGetLastError();  // pageable: not an error for the caller
        return nullptr;
    }
    if (a.type != hipMemoryTypeHost || b.type != hipMemoryTypeHost || a.device != device || !a.devicePointer ||
        !b.devicePointer || (uint8_t*)b.devicePointer - (uint8_t*)a.devicePointer != (ptrdiff_t)(len - 1))
        return nullptr;
    return (uint8_t*)a.devicePointer;
}

// Tuning (A/B runs): lost_disk_fast = false disables the optimistic
// lost-disk GET/heal order, zero_copy = false the in-place kernels on pinned
// blocks.
bool lost_disk_fast_enabled() { return rsg::tuning().lost_disk_fast; }
bool zero_copy_enabled() { return rsg::tuning().zero_copy; }

// Device-batch calls run on the caller's stream; NULL is the HIP null (default)
// stream, which is also torch's default stream, so ordering with the caller holds.
hipStream_t pick_stream(rsg_ctx*, void* s) { return (hipStream_t)s; }
}  // namespace

extern "C" {

int rsg_abi_version(void) { return RSG_ABI_VERSION; }

const char* rsg_strerror(int status) {
    switch (status) {
        case RSG_OK: return "ok";
        case RSG_ERR_INVALID_ARG: return "invalid argument";
        case RSG_ERR_ZERO_DATA_SHARDS: return "data_shards must be greater than zero";
        case RSG_ERR_ZERO_PARITY_SHARDS: return "Reed-Solomon encode failed: TooFewParityShards";
        case RSG_ERR_TOO_MANY_SHARDS: return "modern codec does not support this shard count (data + parity > 256)";
        case RSG_ERR_INVALID_SHARD_COUNT: return "invalid shard count";
        case RSG_ERR_INCONSISTENT_LENGTH: return "inconsistent shard length";
        case RSG_ERR_EMPTY_SHARD: return "Reed-Solomon encode failed: EmptyShard";
        case RSG_ERR_TOO_FEW_SHARDS: return "Reed-Solomon reconstruct failed: TooFewShardsPresent";
        case RSG_ERR_NO_VALID_SHARDS: return "No valid shards found";
        case RSG_ERR_INCONSISTENT_SOURCES: return "inconsistent read source shards";
        case RSG_ERR_BITROT_MISMATCH: return "bitrot hash mismatch";
        case RSG_ERR_NO_DEVICE: return "no HIP device";
        case RSG_ERR_DEVICE: return "HIP runtime error";
        case RSG_ERR_OUT_OF_MEMORY: return "out of device memory";
        case RSG_ERR_UNSUPPORTED: return "unsupported configuration";
        case RSG_ERR_FILE_SIZE_MISMATCH: return "bitrot shard file size mismatch";
        case RSG_ERR_UNEXPECTED_EOF: return "unexpected end of file";
        case RSG_ERR_TRAILING_DATA: return "bitrot shard file has trailing data";
    }
    return "unknown rsgpu status";
}

int rsg_device_count(int* count) {
    if (!count) return RSG_ERR_INVALID_ARG;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    *count = (e == hipSuccess) ? n : 0;
    return e == hipSuccess ? RSG_OK : RSG_ERR_NO_DEVICE;
}

int rsg_create(int device, rsg_ctx** out) {
    if (!out) return RSG_ERR_INVALID_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return RSG_ERR_NO_DEVICE;
    if (hipSetDevice(device) != hipSuccess) return RSG_ERR_NO_DEVICE;
    auto* c = new rsg_ctx();
    c->device = device;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return hip_status(e);
    }
    *out = c;
    return RSG_OK;
}

void rsg_destroy(rsg_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) {
        (void)hipStreamSynchronize(ctx->stream);
        (void)hipStreamDestroy(ctx->stream);
    }
    // tickets never waited on: their work drains before anything is freed
    // (a record job's finishing step then releases its scratch)
    std::vector<uint64_t> pending;
    {
        std::lock_guard<std::mutex> g(ctx->pipe_mu);
        for (auto& j : ctx->jobs) pending.push_back(j.first);
    }
    for (uint64_t t : pending) (void)rsg_wait(ctx, t);
    for (HostLane& l : ctx->lanes) {
        if (l.stream) {
            (void)hipStreamSynchronize(l.stream);
            (void)hipStreamDestroy(l.stream);
        }
        if (l.d_buf) (void)hipFree(l.d_buf);
    }
    for (int i = 0; i < rsg_ctx::kPipeSlots; ++i) {
        if (ctx->pipe_stream[i]) {
            (void)hipStreamSynchronize(ctx->pipe_stream[i]);
            (void)hipStreamDestroy(ctx->pipe_stream[i]);
        }
        if (ctx->d_stage[i]) (void)hipFree(ctx->d_stage[i]);
    }
    ctx->jobs.clear();  // events destroyed with the last reference
    ctx->rec_free.clear();
    delete ctx;
}

int rsg_check_geometry(int k, int m) { return check_geometry(k, m); }

int rsg_pin(void* ptr, size_t bytes) {
    if (!ptr || !bytes) return RSG_ERR_INVALID_ARG;
    return hip_status(hipHostRegister(ptr, bytes, hipHostRegisterDefault));
}

int rsg_unpin(void* ptr) {
    if (!ptr) return RSG_ERR_INVALID_ARG;
    return hip_status(hipHostUnregister(ptr));
}

// Host-memory batch encode (the PUT path: encode_batched's producer,
// encode.rs:795-919), asynchronous.  Sub-batches of `chunk` stripes go
// round-robin over the context's kPipeSlots stream/staging pairs: H2D of the
// data shards (one 2-D copy), encode (+ fused digests), D2H of parity (+
// digests); the copy engines of one slot overlap the kernels of the others,
// and the sub-batches of consecutive jobs keep the link busy back to back.
// The ticket completes when every sub-batch has landed in host memory; the
// caller keeps h_stripes / h_digests alive and untouched until then (the
// reference's EncodedBlock owns its Bytes the same way, encode.rs:64-72).
int rsg_encode_batch_host_submit(rsg_ctx* ctx, int k, int m, size_t shard_len, size_t n, uint8_t* h_stripes,
                                 size_t shard_pitch, size_t stripe_stride, uint8_t* h_digests, int algo,
                                 uint64_t* ticket) {
    int st = enter(ctx);
    if (st) return st;
    if (!ticket) return RSG_ERR_INVALID_ARG;
    *ticket = 0;
    if ((st = check_geometry(k, m))) return st;
    if (n && !h_stripes) return RSG_ERR_INVALID_ARG;
    if (shard_pitch < shard_len) return RSG_ERR_INCONSISTENT_LENGTH;
    if (stripe_stride < (size_t)(k + m) * shard_pitch) return RSG_ERR_INVALID_ARG;
    const bool want_hash = h_digests && algo != RSG_HASH_NONE;
    if (want_hash && !hash_key(algo)) return RSG_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> g(ctx->pipe_mu);
    auto job = std::make_shared<rsg_ctx::Job>();
    // nothing to move: parity of m = 0 is empty; digests are still computed
    // (an empty shard hashes to the digest of the empty message)
    const bool work = n > 0 && ((m > 0 && shard_len > 0) || want_hash);
    if (work) {
        // device layout: compact a3 stripes, 256-B aligned shards
        const uint64_t dpitch = std::max<uint64_t>(256, round_up(shard_len, 256));
        const uint64_t dstride = dpitch * (k + m);
        const uint64_t target = 96ull << 20;  // ~96 MiB per sub-batch
        const uint64_t chunk = std::max<uint64_t>(1, std::min<uint64_t>(n, target / dstride));
        const uint64_t dig_bytes = want_hash ? chunk * (k + m) * 32 : 0;
        if ((st = ctx->ensure_pipeline((size_t)(chunk * dstride + dig_bytes)))) return st;
        const size_t dpitch_data = (shard_pitch == dpitch) ? (size_t)(k * dpitch) : 0;
        bool used[rsg_ctx::kPipeSlots] = {};
        const int fail_at = ctx->fail_subbatch.load();  // rsg_test_fail_subbatch (tests only)
        int sub = 0;
        for (uint64_t s0 = 0; s0 < n && !st; s0 += chunk, ++sub) {
            const int b = (int)(ctx->next_slot++ % rsg_ctx::kPipeSlots);
            used[b] = true;
            hipStream_t s = ctx->pipe_stream[b];
            const uint64_t cnt = std::min<uint64_t>(chunk, n - s0);
            uint8_t* hbase = h_stripes + s0 * stripe_stride;
            uint8_t* d = ctx->d_stage[b];
            if (shard_len == 0) {
            } else if (dpitch_data) {  // data shards contiguous per stripe on both sides
                st = hip_status(hipMemcpy2DAsync(d, dstride, hbase, stripe_stride, dpitch_data, cnt,
                                                 hipMemcpyHostToDevice, s));
            } else {
                for (int i = 0; i < k && !st; ++i)
                    st = hip_status(hipMemcpy2DAsync(d + i * dpitch, dstride, hbase + i * shard_pitch,
                                                     stripe_stride, shard_len, cnt, hipMemcpyHostToDevice, s));
            }
            uint8_t* ddig = want_hash ? d + chunk * dstride : nullptr;
            if (!st && sub == fail_at) st = RSG_ERR_DEVICE;  // fault injection (tests only)
            if (!st) st = rsg_encode_batch_dev(ctx, k, m, shard_len, cnt, d, dpitch, dstride, ddig, algo, s);
            for (int p = 0; p < m && shard_len && !st; ++p)
                st = hip_status(hipMemcpy2DAsync(hbase + (k + p) * shard_pitch, stripe_stride, d + (k + p) * dpitch,
                                                 dstride, shard_len, cnt, hipMemcpyDeviceToHost, s));
            if (!st && want_hash)
                st = hip_status(hipMemcpyAsync(h_digests + s0 * (k + m) * 32, ddig, cnt * (k + m) * 32,
                                               hipMemcpyDeviceToHost, s));
        }
        if (st) {
            // An enqueue failed after earlier sub-batches were queued: their
            // copies still read h_stripes and write parity / digests into the
            // caller's buffers.  Drain every slot this job used before
            // returning the error, so no copy outlives the call (the caller
            // gets no ticket and may free the buffers at once).
            for (int b = 0; b < rsg_ctx::kPipeSlots; ++b)
                if (used[b]) (void)hipStreamSynchronize(ctx->pipe_stream[b]);
            return st;
        }
        for (int b = 0; b < rsg_ctx::kPipeSlots && !st; ++b) {
            if (!used[b]) continue;
            hipEvent_t e;
            if ((st = hip_status(hipEventCreateWithFlags(&e, hipEventDisableTiming)))) break;
            job->done.push_back(e);
            st = hip_status(hipEventRecord(e, ctx->pipe_stream[b]));
        }
        if (st) {  // no ticket: drain the queued sub-batches here (as above)
            for (int b = 0; b < rsg_ctx::kPipeSlots; ++b)
                if (used[b]) (void)hipStreamSynchronize(ctx->pipe_stream[b]);
            return st;
        }
    }
    *ticket = ctx->next_ticket++;
    ctx->jobs.emplace(*ticket, std::move(job));
    return RSG_OK;
}

namespace {
// Query (wait = false) or finish (wait = true) a ticket; a finished ticket is
// released.  *done = 1 once every sub-batch of the job has completed.
// Several threads may wait on or poll one ticket: each holds a reference to
// the job, so its events outlive every waiter; all of them see it finish,
// and the ticket is unknown (RSG_ERR_INVALID_ARG) only to calls made after.
int finish_ticket(rsg_ctx* ctx, uint64_t ticket, bool wait, int* done) {
    int st = enter(ctx);
    if (st) return st;
    if (done) *done = 0;
    std::shared_ptr<rsg_ctx::Job> job;
    {
        std::lock_guard<std::mutex> g(ctx->pipe_mu);
        auto it = ctx->jobs.find(ticket);
        if (it == ctx->jobs.end()) return RSG_ERR_INVALID_ARG;
        job = it->second;
    }
    int res = RSG_OK;
    for (hipEvent_t e : job->done) {
        const hipError_t q = wait ? hipEventSynchronize(e) : hipEventQuery(e);
        if (q == hipErrorNotReady) {  // still in flight (poll only)
            // hipEventQuery's "not ready" is recorded as the thread's last
            // error: clear exactly that, so the next launch check does not
            // fail on it, and leave any other pending error in place
            if (hipPeekAtLastError() == hipErrorNotReady) (void)hipGetLastError();
            return RSG_OK;
        }
        if (q != hipSuccess && !res) res = hip_status(q);
    }
    {  // a record job's host finishing step, exactly once
        std::lock_guard<std::mutex> g(job->fin_mu);
        if (!job->finished) {
            job->result = job->finish ? job->finish(res) : res;
            job->finish = nullptr;  // releases the job's scratch
            job->finished = true;
        }
        res = job->result;
    }
    {
        std::lock_guard<std::mutex> g(ctx->pipe_mu);
        auto it = ctx->jobs.find(ticket);
        if (it != ctx->jobs.end() && it->second == job) ctx->jobs.erase(it);
    }
    if (done) *done = 1;
    return res;
}
}  // namespace

int rsg_poll(rsg_ctx* ctx, uint64_t ticket, int* done) {
    if (!done) return RSG_ERR_INVALID_ARG;
    return finish_ticket(ctx, ticket, false, done);
}

int rsg_wait(rsg_ctx* ctx, uint64_t ticket) { return finish_ticket(ctx, ticket, true, nullptr); }

int rsg_encode_batch_host(rsg_ctx* ctx, int k, int m, size_t shard_len, size_t n, uint8_t* h_stripes,
                          size_t shard_pitch, size_t stripe_stride, uint8_t* h_digests, int algo) {
    uint64_t t = 0;
    int st = rsg_encode_batch_host_submit(ctx, k, m, shard_len, n, h_stripes, shard_pitch, stripe_stride, h_digests,
                                          algo, &t);
    if (st) return st;
    return rsg_wait(ctx, t);
}

int rsg_matrix(int k, int m, uint8_t* out) {
    if (!out) return RSG_ERR_INVALID_ARG;
    int st = check_geometry(k, m);
    if (st) return st;
    if (m == 0) return RSG_ERR_ZERO_PARITY_SHARDS;
    auto cd = get_codec(k, m);
    if (!cd) return RSG_ERR_INVALID_ARG;
    std::memcpy(out, cd->matrix.data(), cd->matrix.size());
    return RSG_OK;
}

int rsg_sync(rsg_ctx* ctx, void* stream) {
    int st = enter(ctx);
    if (st) return st;
    return hip_status(hipStreamSynchronize(pick_stream(ctx, stream)));
}

// ---- device-batch API ----

int rsg_encode_batch_dev(rsg_ctx* ctx, int k, int m, size_t shard_len, size_t n, uint8_t* d_stripes,
                         size_t shard_pitch, size_t stripe_stride, uint8_t* d_digests, int algo, void* stream) {
    int st = enter(ctx);
    if (st) return st;
    if ((st = check_geometry(k, m))) return st;
    if (n && !d_stripes) return RSG_ERR_INVALID_ARG;
    if (shard_pitch < shard_len) return RSG_ERR_INCONSISTENT_LENGTH;
    hipStream_t s = pick_stream(ctx, stream);
    const bool want_hash = d_digests && algo != RSG_HASH_NONE;
    if (want_hash && !hash_key(algo)) return RSG_ERR_INVALID_ARG;
    // the fused kernels take any shard length and alignment (the launcher
    // picks one whose requirements the layout meets)
    if (want_hash && m > 0 && n > 0 && shard_len > 0 && fused_enabled() && rsg::fused_supported(k, m, shard_len)) {
        // one pass: parity + all k+m digests (rs_kernels.hip k_encode_hash_fused)
        auto cd = get_codec(k, m);
        if (!cd) return RSG_ERR_INVALID_ARG;
        RowSet rs = encode_rows(*cd, shard_pitch);
        rsg::GfApplyParams p;
        fill_params(rs, 0, 0, d_stripes, d_stripes, stripe_stride, stripe_stride, rsg::GF_MODE_STORE, nullptr, p);
        rsg::HashParams h;
        std::memset(&h, 0, sizeof(h));
        std::memcpy(h.key, hash_key(algo), sizeof(h.key));
        h.out = d_digests;
        return hip_status(rsg::launch_encode_hash_fused(p, h, shard_len, n, s));
    }
    if (m > 0 && shard_len > 0) {
        auto cd = get_codec(k, m);
        if (!cd) return RSG_ERR_INVALID_ARG;
        RowSet rs = encode_rows(*cd, shard_pitch);
        st = apply_rows(rs, d_stripes, d_stripes, stripe_stride, stripe_stride, shard_len, n, rsg::GF_MODE_STORE,
                        nullptr, s);
        if (st) return st;
    }
    if (want_hash) {
        st = hash_messages(algo, d_stripes, shard_len, n * (uint64_t)(k + m), (uint64_t)(k + m), shard_pitch,
                           stripe_stride, d_digests, s);
        if (st) return st;
    }
    return RSG_OK;
}

int rsg_reconstruct_batch_dev(rsg_ctx* ctx, int k, int m, size_t shard_len, size_t n, uint8_t* d_stripes,
                              size_t shard_pitch, size_t stripe_stride, const uint8_t* present, int mode,
                              void* stream) {
    int st = enter(ctx);
    if (st) return st;
    if ((st = check_geometry(k, m))) return st;
    if (!present || (n && !d_stripes)) return RSG_ERR_INVALID_ARG;
    if (mode < RSG_RECONSTRUCT_DATA || mode > RSG_RECONSTRUCT_REENCODE_PARITY) return RSG_ERR_INVALID_ARG;
    int npresent = 0;
    for (int i = 0; i < k + m; ++i) npresent += present[i] ? 1 : 0;
    if (npresent < k) return RSG_ERR_TOO_FEW_SHARDS;
    if (m == 0 || shard_len == 0 || n == 0) return RSG_OK;
    if (npresent == k + m && mode != RSG_RECONSTRUCT_REENCODE_PARITY) return RSG_OK;
    auto cd = get_codec(k, m);
    if (!cd) return RSG_ERR_INVALID_ARG;
    auto plan = cd->plan(present);
    if (!plan) return RSG_ERR_TOO_FEW_SHARDS;
    RowSet rs = reconstruct_rows(*cd, *plan, present, mode, shard_pitch);
    return apply_rows(rs, d_stripes, d_stripes, stripe_stride, stripe_stride, shard_len, n, rsg::GF_MODE_STORE,
                      nullptr, pick_stream(ctx, stream));
}

int rsg_verify_batch_dev(rsg_ctx* ctx, int k, int m, size_t shard_len, size_t n, const uint8_t* d_stripes,
                         size_t shard_pitch, size_t stripe_stride, uint8_t* d_ok, void* stream) {
    int st = enter(ctx);
    if (st) return st;
    if ((st = check_geometry(k, m))) return st;
    if (n && (!d_stripes || !d_ok)) return RSG_ERR_INVALID_ARG;
    hipStream_t s = pick_stream(ctx, stream);
    if (n == 0) return RSG_OK;
    if ((st = hip_status(hipMemsetAsync(d_ok, 1, n, s)))) return st;
    if (m == 0 || shard_len == 0) return RSG_OK;
    auto cd = get_codec(k, m);
    if (!cd) return RSG_ERR_INVALID_ARG;
    RowSet rs = encode_rows(*cd, shard_pitch);
    return apply_rows(rs, d_stripes, const_cast<uint8_t*>(d_stripes), stripe_stride, stripe_stride, shard_len, n,
                      rsg::GF_MODE_COMPARE, d_ok, s);
}

int rsg_hash_batch_dev(rsg_ctx* ctx, int algo, const uint8_t* d_data, size_t len, size_t stride, size_t n,
                       uint8_t* d_out, void* stream) {
    int st = enter(ctx);
    if (st) return st;
    if (n && (!d_out || (len && !d_data))) return RSG_ERR_INVALID_ARG;
    if (!hash_key(algo)) return RSG_ERR_INVALID_ARG;
    return hash_messages(algo, d_data, len, n, 1, 0, stride, d_out, pick_stream(ctx, stream));
}

// GET-side engine: verify every [digest][block] record, then serve or rebuild
// the data shards of each stripe, runs of stripes with one erasure pattern at
// a time (normally one run: whole shard files present or absent).
}  // extern "C"

namespace {

// Hash `count` record files' n records in place: digest written into each
// record's 32-byte header (BitrotWriter::write framing).
int hash_records_inplace(uint8_t* const* files, int count, uint64_t shard_len, uint64_t n, const uint64_t* key,
                         hipStream_t s) {
    std::vector<uint8_t*> f;
    for (int i = 0; i < count; ++i)
        if (files[i]) f.push_back(files[i]);
    for (size_t g0 = 0; g0 < f.size(); g0 += rsg::kMaxHashBases) {
        const size_t g1 = std::min(f.size(), g0 + (size_t)rsg::kMaxHashBases);
        rsg::HashParams h;
        std::memset(&h, 0, sizeof(h));
        h.len = shard_len;
        h.n = (g1 - g0) * n;
        h.stripe_stride = 32 + shard_len;
        std::memcpy(h.key, key, sizeof(h.key));
        h.nbases = (uint32_t)(g1 - g0);
        h.per_base = n;
        h.digest_off = -32;
        for (size_t x = g0; x < g1; ++x) h.base[x - g0] = f[x] + 32;
        int st = hip_status(rsg::launch_hh256(h, s));
        if (st) return st;
    }
    return RSG_OK;
}

// True when every stripe's verified map is exactly `present` (the assumed
// pattern): present rows all ones, absent rows all zeros — a memchr per row
// instead of the per-stripe run scan.
bool flags_match_pattern(const uint8_t* flags, const std::vector<uint8_t>& present, uint64_t n) {
    for (size_t i = 0; i < present.size(); ++i) {
        const uint8_t* row = flags + i * n;
        if (present[i] ? std::memchr(row, 0, n) != nullptr : std::memchr(row, 1, n) != nullptr) return false;
    }
    return true;
}

// Calls f(s0, s1, present) for each maximal run of stripes sharing one
// verified-shard pattern (degraded stripes come in long runs: a lost disk).
template <class F>
int for_each_pattern_run(int t, uint64_t n, const std::vector<uint8_t>& flags, F&& f) {
    std::vector<uint8_t> present(t);
    for (uint64_t s0 = 0; s0 < n;) {
        for (int i = 0; i < t; ++i) present[i] = flags[(size_t)i * n + s0];
        uint64_t s1 = s0 + 1;
        for (; s1 < n; ++s1) {
            bool same = true;
            for (int i = 0; i < t && same; ++i) same = flags[(size_t)i * n + s1] == present[i];
            if (!same) break;
        }
        int st = f(s0, s1, present);
        if (st) return st;
        s0 = s1;
    }
    return RSG_OK;
}

// Verify (and optionally gather) records of the shard files listed in `idx`
// for stripes [lo, hi): flags[i*n + s] in device scratch is set to 1 for a
// present shard and cleared by the kernel on a digest mismatch.  With d_out,
// data shard i's record bodies are also copied to d_out + s*k*S + i*S.
int launch_verify_group(const std::vector<int>& idx, const uint8_t* const* d_files, uint8_t* d_flags, int k,
                        uint64_t shard_len, uint64_t n, uint64_t lo, uint64_t hi, const uint64_t* key,
                        uint8_t* d_out, hipStream_t s) {
    const uint64_t rec = 32 + shard_len;
    int st;
    if (lo == 0 && hi == n) {  // whole flag rows: one memset per run of consecutive files
        for (size_t a = 0; a < idx.size();) {
            size_t b = a + 1;
            while (b < idx.size() && idx[b] == idx[b - 1] + 1) ++b;
            if ((st = hip_status(hipMemsetAsync(d_flags + (size_t)idx[a] * n, 1, (b - a) * n, s)))) return st;
            a = b;
        }
    } else {
        for (int i : idx)
            if ((st = hip_status(hipMemsetAsync(d_flags + (size_t)i * n + lo, 1, hi - lo, s)))) return st;
    }
    for (size_t g0 = 0; g0 < idx.size(); g0 += rsg::kMaxHashBases) {
        const size_t g1 = std::min(idx.size(), g0 + (size_t)rsg::kMaxHashBases);
        rsg::HashParams h;
        std::memset(&h, 0, sizeof(h));
        h.len = shard_len;
        h.per_base = hi - lo;
        h.n = (g1 - g0) * h.per_base;
        h.stripe_stride = rec;
        std::memcpy(h.key, key, sizeof(h.key));
        h.nbases = (uint32_t)(g1 - g0);
        h.digest_off = -32;
        h.copy_stride = (uint64_t)k * shard_len;
        for (size_t x = g0; x < g1; ++x) {
            const int i = idx[x];
            h.base[x - g0] = d_files[i] + lo * rec + 32;
            h.flag_base[x - g0] = d_flags + (size_t)i * n + lo;
            if (d_out && i < k) h.copy_base[x - g0] = d_out + lo * h.copy_stride + (uint64_t)i * shard_len;
        }
        if ((st = hip_status(rsg::launch_hh256(h, s)))) return st;
    }
    return RSG_OK;
}

// One multi-file hash launch (per kMaxHashBases files) that verifies the
// records of the files in `idx` (flags[i*n + s] cleared on a mismatch; the
// caller sets the present rows to 1 first) and writes the digest header of
// every record of every non-null target file (BitrotWriter framing).
int launch_verify_and_digest(const std::vector<int>& idx, const uint8_t* const* d_files, uint8_t* d_flags,
                             uint8_t* const* d_targets, int t, uint64_t shard_len, uint64_t n, const uint64_t* key,
                             hipStream_t s) {
    const uint64_t rec = 32 + shard_len;
    int st;
    for (size_t a = 0; a < idx.size();) {  // present rows to 1: one memset per run of consecutive files
        size_t b = a + 1;
        while (b < idx.size() && idx[b] == idx[b - 1] + 1) ++b;
        if ((st = hip_status(hipMemsetAsync(d_flags + (size_t)idx[a] * n, 1, (b - a) * n, s)))) return st;
        a = b;
    }
    std::vector<std::pair<uint8_t*, uint8_t*>> list;  // (record 0 body, flag row or null = write digest)
    for (int i : idx) list.push_back({const_cast<uint8_t*>(d_files[i]) + 32, d_flags + (size_t)i * n});
    for (int i = 0; i < t; ++i)
        if (d_targets[i]) list.push_back({d_targets[i] + 32, nullptr});
    for (size_t g0 = 0; g0 < list.size(); g0 += rsg::kMaxHashBases) {
        const size_t g1 = std::min(list.size(), g0 + (size_t)rsg::kMaxHashBases);
        rsg::HashParams h;
        std::memset(&h, 0, sizeof(h));
        h.len = shard_len;
        h.per_base = n;
        h.n = (g1 - g0) * n;
        h.stripe_stride = rec;
        std::memcpy(h.key, key, sizeof(h.key));
        h.nbases = (uint32_t)(g1 - g0);
        h.digest_off = -32;
        for (size_t x = g0; x < g1; ++x) {
            h.base[x - g0] = list[x].first;
            h.flag_base[x - g0] = list[x].second;
        }
        if ((st = hip_status(rsg::launch_hh256(h, s)))) return st;
    }
    return RSG_OK;
}

// Device bytes -> host through the call's page-locked mirror, stream
// synchronised on return.
int flags_to_host(RecScratch& sc, const uint8_t* d_src, size_t bytes, uint8_t* dst, hipStream_t s) {
    int st;
    if ((st = sc.ensure(0, bytes))) return st;
    if ((st = hip_status(hipMemcpyAsync(sc.h, d_src, bytes, hipMemcpyDeviceToHost, s)))) return st;
    if ((st = hip_status(hipStreamSynchronize(s)))) return st;
    std::memcpy(dst, sc.h, bytes);
    return RSG_OK;
}

uint64_t rel(const uint8_t* p, const uint8_t* base) { return (uint64_t)(uintptr_t)p - (uint64_t)(uintptr_t)base; }

// Where a GET puts data shard i of stripe s: the gather form's contiguous
// output (n x k*S, every data shard: rsg_decode_records_dev), or the in-place
// form's per-shard target buffers (rsg_decode_records_into_dev: like
// reconstruct_into, only the shards no verified record serves are written).
struct GetOut {
    uint8_t* d_out = nullptr;
    std::vector<uint8_t*> tg;  // in-place form: k targets
    uint64_t tstride = 0, S = 0, ks = 0;
    bool into() const { return !tg.empty(); }
    uint8_t* at(int i, uint64_t s) const { return into() ? tg[i] + s * tstride : d_out + s * ks + (uint64_t)i * S; }
    uint64_t stride() const { return into() ? tstride : ks; }
};

// One record-engine call (GET or heal) between its submit and its finish.
// submit (get_begin / heal_begin) enqueues the optimistic pass — the one the
// call normally needs alone — and the copy of its verdicts into the call's
// page-locked scratch; the ticket's event follows that copy.  finish
// (get_finish / heal_finish), on the first wait or poll that sees the event
// complete, reads the verdicts, redoes the rare runs of stripes whose
// verified pattern differs from the assumed one and fills the caller's
// status array.  The scratch goes back to the context's pool with the job.
struct RecJob {
    rsg_ctx* ctx = nullptr;
    bool heal = false;
    int k = 0, m = 0, t = 0;
    uint64_t S = 0, n = 0, rec = 0;
    const uint64_t* key = nullptr;
    bool verify_surplus = false;
    std::vector<const uint8_t*> files;  // t entries (null: unavailable)
    std::vector<uint8_t*> targets;      // heal: t entries (null: no writer)
    GetOut out;                         // GET
    int* h_status = nullptr;
    uint8_t* h_src = nullptr;  // GET in-place form, optional: [k][n], 1 = served from its record
    hipStream_t s = nullptr;
    std::unique_ptr<RecScratch> sc;
    hipEvent_t fin = nullptr;  // the finishing step's own work (redo runs), when it has any
    std::shared_ptr<Codec> cd;
    enum Phase { GENERAL, FAST, DATA_VERIFIED } phase = GENERAL;
    bool one_pass = false, any_verify = false;
    std::vector<uint8_t> present0;

    uint8_t* d_flags() const { return sc->d; }
    uint8_t* d_ok() const { return sc->d + (size_t)t * n; }
    ~RecJob() {
        if (fin) (void)hipEventDestroy(fin);
        if (sc) ctx->give_scratch(std::move(sc));
    }
    // wait for the work this finishing step queued (not for whatever the
    // caller queued on the stream after the job)
    int drain() {
        int st;
        if (!fin && (st = hip_status(hipEventCreateWithFlags(&fin, hipEventDisableTiming)))) return st;
        if ((st = hip_status(hipEventRecord(fin, s)))) return st;
        return hip_status(hipEventSynchronize(fin));
    }
    void collect_time() {
        if (sc->timing) ctx->last_kernel_ms.store(sc->tsum());
    }
};

// One-pass GET/heal (k_decode_records_dma) for a batch of n stripes.  A
// workgroup walks its 8 stripes front to back (~0.6 ms for 1 MiB RS(8,4)
// stripes), so below ~1024 stripes, where the grid does not fill the CUs,
// the two-pass path (GF pass spread over every column, then one verify
// launch) returns sooner: n = 8 takes 0.67 ms one-pass.  The context's
// record-engine setting (rsg_set_record_engine: tests and A/B runs) forces
// either path.
bool get_dma_enabled(const rsg_ctx* ctx, uint64_t n) {
    const int e = ctx->record_engine.load();
    if (e == RSG_RECORD_ENGINE_ONE_PASS) return true;
    if (e == RSG_RECORD_ENGINE_TWO_PASS) return false;
    return n >= 1024;
}

// Every present record of every stripe verified in one launch (gathering the
// present data into d_out when given); flags returns the verified map
// [shard][stripe].  Synchronous.
int verify_all(RecJob& j, uint8_t* d_out, std::vector<uint8_t>& flags) {
    int st;
    if ((st = hip_status(hipMemsetAsync(j.d_flags(), 0, (size_t)j.t * j.n, j.s)))) return st;
    std::vector<int> all_idx;
    for (int i = 0; i < j.t; ++i)
        if (j.files[i]) all_idx.push_back(i);
    j.sc->tmark(j.s);
    if ((st = launch_verify_group(all_idx, j.files.data(), j.d_flags(), j.k, j.S, j.n, 0, j.n, j.key, d_out, j.s))) return st;
    j.sc->tmark(j.s);
    flags.assign((size_t)j.t * j.n, 0);
    return flags_to_host(*j.sc, j.d_flags(), flags.size(), flags.data(), j.s);
}

// GET verify-before-use, first half: the k data records of every stripe
// verified (and gathered into d_out when given) in one launch, their flags
// copied back asynchronously into the scratch mirror [0, k*n); the parity
// rows are cleared on the device.
int verify_data_begin(RecJob& j, uint8_t* d_out) {
    int st;
    if ((st = hip_status(hipMemsetAsync(j.d_flags(), 0, (size_t)j.t * j.n, j.s)))) return st;
    std::vector<int> data_idx;
    for (int i = 0; i < j.k; ++i)
        if (j.files[i]) data_idx.push_back(i);
    j.sc->tmark(j.s);
    if ((st = launch_verify_group(data_idx, j.files.data(), j.d_flags(), j.k, j.S, j.n, 0, j.n, j.key, d_out, j.s)))
        return st;
    j.sc->tmark(j.s);
    return j.sc->copy_back(j.s, j.d_flags(), (size_t)j.k * j.n);
}

// Second half, once the data flags have landed: the parity records are
// verified for the stripes that need them (a data record rotten), and flags
// returns the whole verified map (an unread parity record counts as absent).
int verify_parity_rest(RecJob& j, std::vector<uint8_t>& flags) {
    const int k = j.k, t = j.t;
    const uint64_t n = j.n;
    flags.assign((size_t)t * n, 0);
    std::memcpy(flags.data(), j.sc->h, (size_t)k * n);
    uint64_t lo = n, hi = 0;
    for (uint64_t x = 0; x < n; ++x) {
        bool whole = true;
        for (int i = 0; i < k && whole; ++i) whole = flags[(size_t)i * n + x] != 0;
        if (!whole) {
            lo = std::min(lo, x);
            hi = x + 1;
        }
    }
    std::vector<int> par_idx;
    for (int i = k; i < t; ++i)
        if (j.files[i]) par_idx.push_back(i);
    if (lo >= hi || par_idx.empty()) return RSG_OK;
    int st;
    j.sc->tmark(j.s);
    if ((st = launch_verify_group(par_idx, j.files.data(), j.d_flags(), k, j.S, n, lo, hi, j.key, nullptr, j.s)))
        return st;
    j.sc->tmark(j.s);
    return flags_to_host(*j.sc, j.d_flags() + (size_t)k * n, (size_t)j.m * n, flags.data() + (size_t)k * n, j.s);
}

// Rebuild the missing data of stripes [s0, s1) that share one valid-shard
// pattern from the first k valid shards, read in place from the records, and
// (verify_surplus) compare every other valid parity with its re-derived value
// (erasure.rs:935-973).  With `gather` (gather form only), the present data
// shards are copied to the output by the same pass (copy-through).
int get_rebuild_run(RecJob& j, uint64_t s0, uint64_t s1, const std::vector<uint8_t>& present, bool gather) {
    const int k = j.k, t = j.t;
    const uint64_t rec = j.rec, S = j.S, cnt = s1 - s0;
    int valid = 0, missing_data = 0, e;
    for (int i = 0; i < t; ++i) valid += present[i];
    for (int i = 0; i < k; ++i) missing_data += present[i] ? 0 : 1;
    const int run_status = valid < k ? RSG_ERR_TOO_FEW_SHARDS : RSG_OK;
    for (uint64_t x = s0; x < s1; ++x) j.h_status[x] = run_status;
    if (run_status != RSG_OK) return RSG_OK;
    if (!missing_data) {
        if (!gather) return RSG_OK;  // verified data already gathered / served in place
        for (int i = 0; i < k; ++i)
            if ((e = hip_status(hipMemcpy2DAsync(j.out.at(i, s0), j.out.stride(), j.files[i] + s0 * rec + 32, rec, S,
                                                 cnt, hipMemcpyDeviceToDevice, j.s))))
                return e;
        return RSG_OK;
    }
    auto plan = j.cd->plan(present.data());
    if (!plan) return RSG_ERR_TOO_FEW_SHARDS;
    // survivors read in place from the records; base = first survivor, out =
    // the first missing data shard's slot (every offset relative to them)
    const uint8_t* base = j.files[plan->survivors[0]] + s0 * rec + 32;
    int first_missing = 0;
    while (present[first_missing]) ++first_missing;
    uint8_t* out = j.out.at(first_missing, s0);
    RowSet rs;
    rs.C = k;
    for (int sv : plan->survivors) rs.in_off.push_back(rel(j.files[sv] + s0 * rec + 32, base));
    if (gather) {
        rs.copy.assign(k, 0);
        rs.copy_off.assign(k, 0);
        for (int c = 0; c < k; ++c)
            if (plan->survivors[c] < k) {
                rs.copy[c] = 1;
                rs.copy_off[c] = rel(j.out.at(plan->survivors[c], s0), out);
            }
    }
    for (int i = 0; i < k; ++i) {
        if (present[i]) continue;
        rs.coef.resize((size_t)(rs.R + 1) * k);
        plan_row(*j.cd, *plan, i, &rs.coef[(size_t)rs.R * k]);
        rs.out_off.push_back(rel(j.out.at(i, s0), out));
        ++rs.R;
    }
    // surplus parity must agree with the rebuilt data (erasure.rs:935-973)
    RowSet vs;
    vs.C = k;
    vs.in_off = rs.in_off;
    if (j.verify_surplus && valid > k) {
        for (int p = k; p < t; ++p) {
            if (!present[p] || is_survivor(*plan, p)) continue;  // a survivor re-derives to itself
            vs.coef.resize((size_t)(vs.R + 1) * k);
            plan_row(*j.cd, *plan, p, &vs.coef[(size_t)vs.R * k]);
            vs.out_off.push_back(rel(j.files[p] + s0 * rec + 32, base));
            ++vs.R;
        }
    }
    if (vs.R) j.any_verify = true;
    if (vs.R && rs.R + vs.R <= rsg::kMaxR && k <= rsg::kMaxC) {
        // rebuild + check in one pass over the survivors
        RowSet both = rs;
        both.coef.insert(both.coef.end(), vs.coef.begin(), vs.coef.end());
        for (uint64_t o : vs.out_off) both.out_off.push_back(rel(base + o, out));  // compare targets relative to `out`
        both.R = rs.R + vs.R;
        return apply_store_compare(both, rs.R, base, out, rec, j.out.stride(), rec, S, cnt, j.d_ok() + s0, j.s);
    }
    if ((e = apply_rows(rs, base, out, rec, j.out.stride(), S, cnt, rsg::GF_MODE_STORE, nullptr, j.s))) return e;
    if (!vs.R) return RSG_OK;
    return apply_rows(vs, base, const_cast<uint8_t*>(base), rec, rec, S, cnt, rsg::GF_MODE_COMPARE, j.d_ok() + s0,
                      j.s);
}

// Launch k_decode_records_dma over all stripes for the erasure pattern
// present0: present files in ascending order, the first k are the survivors
// (DecodePlan order); rows = the missing data shards (stored to the GET's
// output), then (with verify_surplus) the present non-survivor parity,
// compared in place.  The gather form also copies the present data through.
int launch_get_one_pass(RecJob& j, const std::vector<int>& files) {
    const int k = j.k;
    auto plan = j.cd->plan(j.present0.data());
    if (!plan) return RSG_ERR_TOO_FEW_SHARDS;
    for (int c = 0; c < k; ++c)
        if (plan->survivors[c] != files[c]) return RSG_ERR_INVALID_ARG;  // survivors = first k present
    std::vector<uint8_t> coef;
    rsg::GfApplyParams p;
    std::memset(&p, 0, sizeof(p));
    int first_missing = 0;
    while (j.present0[first_missing]) ++first_missing;
    p.out_base = j.out.at(first_missing, 0);
    int R = 0;
    for (int i = 0; i < k; ++i) {
        if (j.present0[i]) continue;
        coef.resize((size_t)(R + 1) * k);
        plan_row(*j.cd, *plan, i, &coef[(size_t)R * k]);
        p.out_off[R++] = rel(j.out.at(i, 0), p.out_base);
    }
    const int n_store = R;
    if (j.verify_surplus) {
        for (int f = k; f < (int)files.size(); ++f) {  // present non-survivors: parity, ascending
            if (R >= rsg::kMaxR) return RSG_ERR_UNSUPPORTED;
            coef.resize((size_t)(R + 1) * k);
            plan_row(*j.cd, *plan, files[f], &coef[(size_t)R * k]);
            ++R;
        }
    }
    if (R > (j.m > 4 ? 8 : 4) || R == 0) return RSG_ERR_UNSUPPORTED;
    if (R > n_store) j.any_verify = true;
    for (int r = 0; r < R; ++r)
        for (int c = 0; c < k; ++c) coef_tables(coef[(size_t)r * k + c], p.tab[r][c]);
    p.C = (uint32_t)k;
    p.R = (uint32_t)R;
    p.n_store = (uint32_t)n_store;
    p.mode = rsg::GF_MODE_STORE_COMPARE;
    p.out_stripe_stride = j.out.stride();
    p.ok_flags = j.d_ok();
    if (!j.out.into())
        for (int c = 0; c < k; ++c)
            if (files[c] < k) {
                p.copy_mask |= 1u << c;
                p.copy_off[c] = rel(j.out.at(files[c], 0), p.out_base);
            }
    rsg::HashParams h;
    std::memset(&h, 0, sizeof(h));
    h.len = j.S;
    h.stripe_stride = j.rec;
    std::memcpy(h.key, j.key, sizeof(h.key));
    h.nbases = (uint32_t)files.size();
    h.digest_off = -32;
    for (size_t f = 0; f < files.size(); ++f) {
        h.base[f] = j.files[files[f]] + 32;
        h.flag_base[f] = j.d_flags() + (size_t)files[f] * j.n;
    }
    j.sc->tmark(j.s);  // the timing hook opens after the host-side preparation
    const bool any_table = j.ctx->record_engine.load() == RSG_RECORD_ENGINE_ONE_PASS;  // forced: the table kernel too
    const hipError_t e =
        rsg::launch_decode_records_dma(p, h, k, j.m, (int)files.size(), j.S, j.n, coef.data(), any_table, j.s);
    if (e == hipErrorNotSupported) j.sc->tunmark();
    return e == hipErrorNotSupported ? RSG_ERR_UNSUPPORTED : hip_status(e);  // unsupported: nothing launched
}

// GET submit: the pass the call normally needs alone, then the verdict copy.
//  - a data file missing (a lost disk, the common degraded case): every
//    stripe misses the same data shards, so ONE optimistic pass over the
//    present records rebuilds the missing data (gather form: and copies the
//    present data through), checks the surplus parity and verifies every
//    present record, as if all verify — k_decode_records_dma / _net where the
//    geometry has a one-pass kernel, else a GF pass then a verify launch;
//  - every data file present: one launch verifies the k data records (gather
//    form: copying them to the output); the in-place form writes nothing;
//  - anything else (no codec, too many rows for one pass): the general path,
//    all of it in the finishing step.
int get_begin(RecJob& j) {
    const int k = j.k, m = j.m, t = j.t;
    const uint64_t n = j.n;
    int st;
    if ((st = j.sc->ensure((size_t)(t + 1) * n, (size_t)(t + 1) * n))) return st;
    if (m > 0 && !(j.cd = get_codec(k, m))) return RSG_ERR_INVALID_ARG;
    j.present0.assign(t, 0);
    int nfiles = 0, lost_data = 0;
    std::vector<int> all_idx;
    for (int i = 0; i < t; ++i) {
        j.present0[i] = j.files[i] ? 1 : 0;
        nfiles += j.present0[i];
        if (j.files[i]) all_idx.push_back(i);
        if (i < k && !j.files[i]) ++lost_data;
    }
    const int surplus = std::max(0, nfiles - k);  // present shards beyond the k survivors
    const bool fast = m > 0 && lost_data > 0 && nfiles >= k && k <= rsg::kMaxC &&
                      lost_data + (j.verify_surplus ? surplus : 0) <= rsg::kMaxR && lost_disk_fast_enabled();
    if (fast) {
        j.phase = RecJob::FAST;
        // (record files and slots at any alignment: the ring's LDS-DMA and
        // the kernels' 8-byte stores take unaligned addresses)
        bool one_pass = get_dma_enabled(j.ctx, n) && rsg::decode_dma_supported(k, m, nfiles, j.S);
        if (one_pass) {
            // verify every present record, rebuild (and gather) and check
            // the surplus parity in ONE pass; the kernel writes every present
            // file's flags and, with surplus rows, every stripe's verdict
            // whole (no memsets before it)
            st = launch_get_one_pass(j, all_idx);  // opens the timing mark when it launches
            if (st == RSG_ERR_UNSUPPORTED) {  // no network and the table kernel is the slower path here
                one_pass = false;
                j.any_verify = false;
            } else if (st) {
                return st;
            } else {
                j.sc->tmark(j.s);
                if (!j.any_verify && (st = hip_status(hipMemsetAsync(j.d_ok(), 1, n, j.s)))) return st;
                for (uint64_t x = 0; x < n; ++x) j.h_status[x] = RSG_OK;
            }
        }
        j.one_pass = one_pass;
        if (!one_pass) {
            if ((st = hip_status(hipMemsetAsync(j.d_ok(), 1, n, j.s)))) return st;
            j.sc->tmark(j.s);
            if ((st = get_rebuild_run(j, 0, n, j.present0, !j.out.into()))) return st;
            j.sc->tmark(j.s);
            if ((st = hip_status(hipMemsetAsync(j.d_flags(), 0, (size_t)t * n, j.s)))) return st;
            j.sc->tmark(j.s);
            if ((st = launch_verify_group(all_idx, j.files.data(), j.d_flags(), k, j.S, n, 0, n, j.key, nullptr, j.s)))
                return st;
            j.sc->tmark(j.s);
        }
        // the verified map and the surplus verdict (adjacent in scratch) in one copy
        return j.sc->copy_back(j.s, j.d_flags(), (size_t)(t + 1) * n);
    }
    if (lost_data == 0) {
        j.phase = RecJob::DATA_VERIFIED;
        if ((st = hip_status(hipMemsetAsync(j.d_ok(), 1, n, j.s)))) return st;
        return verify_data_begin(j, j.out.into() ? nullptr : j.out.d_out);
    }
    j.phase = RecJob::GENERAL;
    return RSG_OK;
}

int get_finish(RecJob& j) {
    const int k = j.k, t = j.t;
    const uint64_t n = j.n;
    const bool gather = !j.out.into();
    std::vector<uint8_t> flags;
    const uint8_t* fmap = nullptr;  // the final verified map [shard][stripe]
    bool queued = false;             // work queued here: drain before returning
    int st;
    if (j.phase == RecJob::FAST) {
        uint8_t* hf = j.sc->h;
        if (j.one_pass)  // absent files' rows were never written on the device
            for (int i = 0; i < t; ++i)
                if (!j.files[i]) std::memset(hf + (size_t)i * n, 0, n);
        bool redone = false;
        if (!flags_match_pattern(hf, j.present0, n)) {
            flags.assign(hf, hf + (size_t)t * n);
            st = for_each_pattern_run(t, n, flags, [&](uint64_t s0, uint64_t s1, const std::vector<uint8_t>& present) {
                if (present == j.present0) return (int)RSG_OK;  // the optimistic pass was right
                redone = true;
                int e = hip_status(hipMemsetAsync(j.d_ok() + s0, 1, s1 - s0, j.s));
                return e ? e : get_rebuild_run(j, s0, s1, present, gather);
            });
            if (st) return st;
        }
        if (!redone) {
            if (j.any_verify)
                for (uint64_t x = 0; x < n; ++x)
                    if (j.h_status[x] == RSG_OK && !hf[(size_t)t * n + x]) j.h_status[x] = RSG_ERR_INCONSISTENT_SOURCES;
            if (j.h_src)
                for (int i = 0; i < k; ++i) std::memcpy(j.h_src + (size_t)i * n, hf + (size_t)i * n, n);
            j.collect_time();
            return RSG_OK;  // nothing queued after the ticket's event
        }
        fmap = flags.data();
        queued = true;
    } else {
        if (j.phase == RecJob::DATA_VERIFIED) {
            if (!std::memchr(j.sc->h, 0, (size_t)k * n)) {  // every data record verified: nothing to rebuild
                for (uint64_t x = 0; x < n; ++x) j.h_status[x] = RSG_OK;
                if (j.h_src) std::memset(j.h_src, 1, (size_t)k * n);
                j.collect_time();
                return RSG_OK;
            }
            if ((st = verify_parity_rest(j, flags))) return st;
        } else {
            if ((st = hip_status(hipMemsetAsync(j.d_ok(), 1, n, j.s)))) return st;
            if ((st = verify_all(j, gather ? j.out.d_out : nullptr, flags))) return st;
        }
        st = for_each_pattern_run(t, n, flags, [&](uint64_t s0, uint64_t s1, const std::vector<uint8_t>& present) {
            return get_rebuild_run(j, s0, s1, present, false);
        });
        if (st) return st;
        fmap = flags.data();
        queued = true;
    }
    if (j.any_verify) {
        std::vector<uint8_t> ok(n, 1);
        if ((st = flags_to_host(*j.sc, j.d_ok(), n, ok.data(), j.s))) return st;
        for (uint64_t x = 0; x < n; ++x)
            if (j.h_status[x] == RSG_OK && !ok[x]) j.h_status[x] = RSG_ERR_INCONSISTENT_SOURCES;
    } else if (queued && (st = j.drain())) {
        return st;
    }
    if (j.h_src)
        for (int i = 0; i < k; ++i) std::memcpy(j.h_src + (size_t)i * n, fmap + (size_t)i * n, n);
    j.collect_time();
    return RSG_OK;
}

// Launch the one-pass heal (k_decode_records_dma with target hashing) for
// the pattern present0: survivors = the first k present files; rows = every
// target (absent from the sources), then the present non-survivor parity,
// compared in place (heal.rs:180-196).
int launch_heal_one_pass(RecJob& j, const std::vector<int>& files, const std::vector<int>& targets) {
    const int k = j.k;
    auto plan = j.cd->plan(j.present0.data());
    if (!plan) return RSG_ERR_TOO_FEW_SHARDS;
    for (int c = 0; c < k; ++c)
        if (plan->survivors[c] != files[c]) return RSG_ERR_INVALID_ARG;
    rsg::GfApplyParams p;
    std::memset(&p, 0, sizeof(p));
    std::vector<uint8_t> coef;
    int R = 0;
    p.out_base = j.targets[targets[0]] + 32;
    for (int i : targets) {
        coef.resize((size_t)(R + 1) * k);
        plan_row(*j.cd, *plan, i, &coef[(size_t)R * k]);
        p.out_off[R++] = rel(j.targets[i] + 32, p.out_base);
    }
    const int n_store = R;
    for (int f = k; f < (int)files.size(); ++f) {  // present non-survivors: parity, ascending
        if (R >= (j.m > 4 ? 8 : 4)) return RSG_ERR_UNSUPPORTED;
        coef.resize((size_t)(R + 1) * k);
        plan_row(*j.cd, *plan, files[f], &coef[(size_t)R * k]);
        ++R;
    }
    if (R > n_store) j.any_verify = true;
    for (int r = 0; r < R; ++r)
        for (int c = 0; c < k; ++c) coef_tables(coef[(size_t)r * k + c], p.tab[r][c]);
    p.C = (uint32_t)k;
    p.R = (uint32_t)R;
    p.n_store = (uint32_t)n_store;
    p.mode = rsg::GF_MODE_STORE_COMPARE;
    p.out_stripe_stride = j.rec;
    p.ok_flags = j.d_ok();
    rsg::HashParams h;
    std::memset(&h, 0, sizeof(h));
    h.len = j.S;
    h.stripe_stride = j.rec;
    std::memcpy(h.key, j.key, sizeof(h.key));
    h.nbases = (uint32_t)files.size();
    h.digest_off = -32;
    for (size_t f = 0; f < files.size(); ++f) {
        h.base[f] = j.files[files[f]] + 32;
        h.flag_base[f] = j.d_flags() + (size_t)files[f] * j.n;
    }
    j.sc->tmark(j.s);  // the timing hook opens after the host-side preparation
    const bool any_table = j.ctx->record_engine.load() == RSG_RECORD_ENGINE_ONE_PASS;  // forced: the table heal too
    const hipError_t e = rsg::launch_heal_records_dma(p, h, k, j.m, (int)files.size(), (int)targets.size(), j.S,
                                                      j.n, coef.data(), any_table, j.s);
    if (e == hipErrorNotSupported) j.sc->tunmark();
    return e == hipErrorNotSupported ? RSG_ERR_UNSUPPORTED : hip_status(e);  // unsupported: nothing launched
}

// Per run of stripes with one verified pattern, ONE pass over the survivors
// (first k verified shards) writes every target's record body — data rebuilt
// or, if verified, reproduced (identity row), parity re-encoded — and
// compares every verified source parity that is not a survivor with its
// re-encoded value: "inconsistent heal source shards" (heal.rs:180-196; a
// survivor parity re-encodes to itself).
int heal_run(RecJob& j, uint64_t s0, uint64_t s1, const std::vector<uint8_t>& present) {
    const int k = j.k, t = j.t;
    const uint64_t rec = j.rec;
    int valid = 0;
    for (int i = 0; i < t; ++i) valid += present[i];
    for (uint64_t x = s0; x < s1; ++x) j.h_status[x] = valid < k ? RSG_ERR_TOO_FEW_SHARDS : RSG_OK;
    if (valid < k) return RSG_OK;
    auto plan = j.cd->plan(present.data());
    if (!plan) return RSG_ERR_TOO_FEW_SHARDS;
    const uint8_t* base = j.files[plan->survivors[0]] + s0 * rec + 32;
    auto off = [&](const uint8_t* p) { return rel(p + s0 * rec + 32, base); };
    RowSet ps, vs;  // target bodies (store), non-survivor verified parity (compare)
    ps.C = vs.C = k;
    for (int sv : plan->survivors) ps.in_off.push_back(off(j.files[sv]));
    vs.in_off = ps.in_off;
    for (int i = 0; i < t; ++i) {
        if (j.targets[i]) {
            ps.coef.resize((size_t)(ps.R + 1) * k);
            plan_row(*j.cd, *plan, i, &ps.coef[(size_t)ps.R * k]);
            ps.out_off.push_back(off(j.targets[i]));
            ++ps.R;
        }
        if (i >= k && present[i] && !is_survivor(*plan, i)) {
            vs.coef.resize((size_t)(vs.R + 1) * k);
            plan_row(*j.cd, *plan, i, &vs.coef[(size_t)vs.R * k]);
            vs.out_off.push_back(off(j.files[i]));
            ++vs.R;
        }
    }
    if (vs.R) j.any_verify = true;
    uint8_t* ob = const_cast<uint8_t*>(base);
    if (ps.R + vs.R <= rsg::kMaxR && k <= rsg::kMaxC) {
        RowSet both = ps;
        both.coef.insert(both.coef.end(), vs.coef.begin(), vs.coef.end());
        both.out_off.insert(both.out_off.end(), vs.out_off.begin(), vs.out_off.end());
        both.R = ps.R + vs.R;
        return apply_store_compare(both, ps.R, base, ob, rec, rec, rec, j.S, s1 - s0, j.d_ok() + s0, j.s);
    }
    int e = apply_rows(ps, base, ob, rec, rec, j.S, s1 - s0, rsg::GF_MODE_STORE, nullptr, j.s);
    if (e || !vs.R) return e;
    return apply_rows(vs, base, ob, rec, rec, j.S, s1 - s0, rsg::GF_MODE_COMPARE, j.d_ok() + s0, j.s);
}

// the target records of stripes [s0, s1) get their HH256S headers
int heal_hash_targets(RecJob& j, uint64_t s0, uint64_t s1) {
    std::vector<uint8_t*> tg(j.t, nullptr);
    for (int i = 0; i < j.t; ++i)
        if (j.targets[i]) tg[i] = j.targets[i] + s0 * j.rec;
    return hash_records_inplace(tg.data(), j.t, j.S, s1 - s0, j.key, j.s);
}

// Heal submit.  Optimistic (replaced disks, sound sources — the common heal):
// one pass writes every target record (body + digest), verifies every source
// record and compares the surplus parity (RS(8,4)/(16,4) networks and the
// k <= 8 table kernel), or a GF pass then one hash launch that verifies the
// sources and writes the targets' digests; then the verified map and the
// parity verdict go back in one copy.  Anything else: the general path, all
// of it in the finishing step.
int heal_begin(RecJob& j) {
    const int k = j.k, m = j.m, t = j.t;
    const uint64_t n = j.n;
    int st;
    if ((st = j.sc->ensure((size_t)(t + 1) * n, (size_t)(t + 1) * n))) return st;
    if (!(j.cd = get_codec(k, m))) return RSG_ERR_INVALID_ARG;
    j.present0.assign(t, 0);
    int valid0 = 0;
    std::vector<int> all_idx, tg_idx;
    for (int i = 0; i < t; ++i) {
        valid0 += (j.present0[i] = j.files[i] ? 1 : 0);
        if (j.files[i]) all_idx.push_back(i);
        if (j.targets[i]) tg_idx.push_back(i);
    }
    if (valid0 < k || !lost_disk_fast_enabled()) {
        j.phase = RecJob::GENERAL;
        return RSG_OK;
    }
    j.phase = RecJob::FAST;
    bool one_pass = get_dma_enabled(j.ctx, n) &&
                    rsg::heal_one_pass_shape(k, m, (int)all_idx.size(), (int)tg_idx.size(), j.S);
    for (int i : tg_idx) one_pass = one_pass && !j.files[i];
    if (one_pass) {
        st = launch_heal_one_pass(j, all_idx, tg_idx);  // opens the timing mark when it launches
        if (st == RSG_ERR_UNSUPPORTED) {  // no network, table heal not preferred for k: the two-pass path
            one_pass = false;
            j.any_verify = false;
        } else if (st) {
            return st;
        } else {
            j.sc->tmark(j.s);
            if (!j.any_verify && (st = hip_status(hipMemsetAsync(j.d_ok(), 1, n, j.s)))) return st;
            for (uint64_t x = 0; x < n; ++x) j.h_status[x] = RSG_OK;
        }
    }
    j.one_pass = one_pass;
    if (!one_pass) {
        if ((st = hip_status(hipMemsetAsync(j.d_ok(), 1, n, j.s)))) return st;
        j.sc->tmark(j.s);
        if ((st = heal_run(j, 0, n, j.present0))) return st;
        j.sc->tmark(j.s);
        if ((st = hip_status(hipMemsetAsync(j.d_flags(), 0, (size_t)t * n, j.s)))) return st;
        j.sc->tmark(j.s);
        if ((st = launch_verify_and_digest(all_idx, j.files.data(), j.d_flags(), j.targets.data(), t, j.S, n, j.key,
                                           j.s)))
            return st;
        j.sc->tmark(j.s);
    }
    return j.sc->copy_back(j.s, j.d_flags(), (size_t)(t + 1) * n);
}

int heal_finish(RecJob& j) {
    const int t = j.t;
    const uint64_t n = j.n, rec = j.rec;
    bool queued = false;
    int st;
    std::vector<uint8_t> flags, ok(n, 1);
    if (j.phase == RecJob::FAST) {
        uint8_t* hf = j.sc->h;
        if (j.one_pass)  // absent files' rows were never written on the device
            for (int i = 0; i < t; ++i)
                if (!j.files[i]) std::memset(hf + (size_t)i * n, 0, n);
        std::memcpy(ok.data(), hf + (size_t)t * n, n);
        bool redone = false;
        if (!flags_match_pattern(hf, j.present0, n)) {
            flags.assign(hf, hf + (size_t)t * n);
            st = for_each_pattern_run(t, n, flags, [&](uint64_t s0, uint64_t s1, const std::vector<uint8_t>& present) {
                if (present == j.present0) return (int)RSG_OK;
                redone = true;
                int e = hip_status(hipMemsetAsync(j.d_ok() + s0, 1, s1 - s0, j.s));
                if (!e) e = heal_run(j, s0, s1, present);
                return e ? e : heal_hash_targets(j, s0, s1);
            });
            if (st) return st;
        }
        if (redone) {
            queued = true;
            if (j.any_verify && (st = flags_to_host(*j.sc, j.d_ok(), n, ok.data(), j.s))) return st;
        }
    } else {
        // verify every source record first (read quorum: k verified shards
        // per stripe), then the per-pattern GF passes, then the digests
        if ((st = hip_status(hipMemsetAsync(j.d_ok(), 1, n, j.s)))) return st;
        if ((st = verify_all(j, nullptr, flags))) return st;
        if ((st = for_each_pattern_run(t, n, flags, [&](uint64_t s0, uint64_t s1, const std::vector<uint8_t>& p) {
                 return heal_run(j, s0, s1, p);
             })))
            return st;
        if ((st = heal_hash_targets(j, 0, n))) return st;
        queued = true;
        if (j.any_verify && (st = flags_to_host(*j.sc, j.d_ok(), n, ok.data(), j.s))) return st;
    }
    if (j.any_verify)
        for (uint64_t x = 0; x < n; ++x)
            if (j.h_status[x] == RSG_OK && !ok[x]) j.h_status[x] = RSG_ERR_INCONSISTENT_SOURCES;
    // A failed stripe's target records hold unverified bytes: their digest
    // headers are zeroed so they can never pass bitrot verification even if a
    // caller ignores h_status (the reference writes nothing for a failed heal).
    for (uint64_t s0 = 0; s0 < n;) {
        if (j.h_status[s0] == RSG_OK) {
            ++s0;
            continue;
        }
        uint64_t s1 = s0 + 1;
        while (s1 < n && j.h_status[s1] != RSG_OK) ++s1;
        for (int i = 0; i < t; ++i)
            if (j.targets[i] && (st = hip_status(hipMemset2DAsync(j.targets[i] + s0 * rec, rec, 0, 32, s1 - s0, j.s))))
                return st;
        queued = true;
        s0 = s1;
    }
    if (queued && (st = j.drain())) return st;
    j.collect_time();
    return RSG_OK;
}

// Register a record job: its event follows the submit's work on the stream;
// the first wait / poll that sees it runs the finishing step.  On a submit
// error nothing of the job stays in flight and no ticket is issued.
int submit_record_job(rsg_ctx* ctx, std::shared_ptr<RecJob> rj, int (*begin)(RecJob&), int (*finish)(RecJob&),
                      uint64_t* ticket) {
    auto job = std::make_shared<rsg_ctx::Job>();
    int st = begin(*rj);
    hipEvent_t e = nullptr;
    if (!st) st = hip_status(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    if (e) job->done.push_back(e);
    if (!st) st = hip_status(hipEventRecord(e, rj->s));
    if (st) {
        (void)hipStreamSynchronize(rj->s);  // the job's queued work reads its scratch
        return st;                          // rj (and its scratch) released here
    }
    job->finish = [rj, finish](int ev) -> int {
        int r = ev ? ev : finish(*rj);
        if (r) (void)hipStreamSynchronize(rj->s);  // nothing of the job outlives its scratch
        rj->sc->tev_used = 0;
        return r;
    };
    std::lock_guard<std::mutex> g(ctx->pipe_mu);
    *ticket = ctx->next_ticket++;
    ctx->jobs.emplace(*ticket, std::move(job));
    return RSG_OK;
}

// A ticket with nothing to wait for (empty batch).
uint64_t done_ticket(rsg_ctx* ctx) {
    std::lock_guard<std::mutex> g(ctx->pipe_mu);
    const uint64_t t = ctx->next_ticket++;
    ctx->jobs.emplace(t, std::make_shared<rsg_ctx::Job>());
    return t;
}

// Byte ranges [a, a+la) and [b, b+lb) intersect.
bool spans_overlap(const uint8_t* a, uint64_t la, const uint8_t* b, uint64_t lb) {
    return (uintptr_t)a < (uintptr_t)b + lb && (uintptr_t)b < (uintptr_t)a + la;
}

// Slots a and b of the in-place GET, stripes at a + s*ts and b + s'*ts (s, s'
// < n), each shard_len bytes: true if some pair of their stripe windows shares
// a byte (two rebuilt shards would be written over each other).  The block
// layout (slot i = base + i*shard_len, ts = k*shard_len) interleaves the
// slots without a collision.
bool slot_windows_collide(const uint8_t* a, const uint8_t* b, uint64_t ts, uint64_t shard_len, uint64_t n) {
    const __int128 d = (__int128)(uintptr_t)b - (__int128)(uintptr_t)a;
    const __int128 t = (__int128)ts;
    __int128 q = d / t;
    if (d % t != 0 && d < 0) q -= 1;  // floor
    for (__int128 c = q; c <= q + 1; ++c) {  // the two stripe offsets nearest to d
        const __int128 diff = d - c * t;
        if ((diff < 0 ? -diff : diff) < (__int128)shard_len && (c < 0 ? -c : c) <= (__int128)n - 1) return true;
    }
    return false;
}

}  // namespace

extern "C" {

int rsg_decode_records_submit(rsg_ctx* ctx, int k, int m, size_t shard_len, size_t n, const uint8_t* const* d_files,
                              int algo, int verify_surplus, uint8_t* d_out, uint8_t* const* d_targets,
                              size_t target_stride, uint8_t* h_src, int* h_status, void* stream, uint64_t* ticket) {
    int st = enter(ctx);
    if (st) return st;
    if (!ticket) return RSG_ERR_INVALID_ARG;
    *ticket = 0;
    if ((st = check_geometry(k, m))) return st;
    if (!d_files || (d_out && d_targets)) return RSG_ERR_INVALID_ARG;  // one output form
    if (n && (!h_status || (!d_out && !d_targets))) return RSG_ERR_INVALID_ARG;
    const uint64_t* key = hash_key(algo);
    if (!key) return RSG_ERR_INVALID_ARG;
    const uint64_t rec = 32 + (uint64_t)shard_len;
    if (d_targets) {
        // in-place form: a slot per data shard (reconstruct_into's shards
        // slice); a slot range overlapping a source record file would be
        // written while it is read
        if (target_stride < shard_len) return RSG_ERR_INVALID_ARG;
        const uint64_t span = n ? (uint64_t)(n - 1) * target_stride + shard_len : 0;
        for (int i = 0; i < k; ++i) {
            if (!d_targets[i]) return RSG_ERR_INVALID_ARG;
            for (int f = 0; f < k + m && span; ++f)
                if (d_files[f] && spans_overlap(d_targets[i], span, d_files[f], (uint64_t)n * rec))
                    return RSG_ERR_INVALID_ARG;
            // two slots whose stripe windows share bytes (one buffer passed
            // as several slots): rebuilt shards would overwrite each other
            for (int j = 0; j < i && n && shard_len; ++j)
                if (slot_windows_collide(d_targets[j], d_targets[i], target_stride, shard_len, n))
                    return RSG_ERR_INVALID_ARG;
        }
    }
    if (n == 0 || shard_len == 0) {
        for (size_t s = 0; s < n; ++s) h_status[s] = RSG_OK;
        if (h_src) std::memset(h_src, 1, (size_t)k * n);
        *ticket = done_ticket(ctx);
        return RSG_OK;
    }
    auto rj = std::make_shared<RecJob>();
    rj->ctx = ctx;
    rj->k = k;
    rj->m = m;
    rj->t = k + m;
    rj->S = shard_len;
    rj->n = n;
    rj->rec = rec;
    rj->key = key;
    rj->verify_surplus = verify_surplus != 0;
    rj->files.assign(d_files, d_files + k + m);
    rj->out.S = shard_len;
    rj->out.ks = (uint64_t)k * shard_len;
    if (d_targets) {
        rj->out.tg.assign(d_targets, d_targets + k);
        rj->out.tstride = target_stride;
    } else {
        rj->out.d_out = d_out;
    }
    rj->h_status = h_status;
    rj->h_src = h_src;
    rj->s = pick_stream(ctx, stream);
    rj->sc = ctx->take_scratch();
    return submit_record_job(ctx, std::move(rj), get_begin, get_finish, ticket);
}

int rsg_decode_records_dev(rsg_ctx* ctx, int k, int m, size_t shard_len, size_t n, const uint8_t* const* d_files,
                           int algo, int verify_surplus, uint8_t* d_out, int* h_status, void* stream) {
    if (!d_out && n) return RSG_ERR_INVALID_ARG;
    uint64_t t = 0;
    int st = rsg_decode_records_submit(ctx, k, m, shard_len, n, d_files, algo, verify_surplus, d_out, nullptr, 0,
                                       nullptr, h_status, stream, &t);
    return st ? st : rsg_wait(ctx, t);
}

int rsg_decode_records_into_dev(rsg_ctx* ctx, int k, int m, size_t shard_len, size_t n,
                                const uint8_t* const* d_files, int algo, int verify_surplus,
                                uint8_t* const* d_targets, size_t target_stride, uint8_t* h_src, int* h_status,
                                void* stream) {
    uint64_t t = 0;
    int st = rsg_decode_records_submit(ctx, k, m, shard_len, n, d_files, algo, verify_surplus, nullptr, d_targets,
                                       target_stride, h_src, h_status, stream, &t);
    return st ? st : rsg_wait(ctx, t);
}

int rsg_set_kernel_timing(rsg_ctx* ctx, int on) {
    int st = enter(ctx);
    if (st) return st;
    ctx->timing.store(on != 0);
    ctx->last_kernel_ms.store(-1.f);
    return RSG_OK;
}

int rsg_test_fail_subbatch(rsg_ctx* ctx, int index) {
    if (!ctx || index < -1) return RSG_ERR_INVALID_ARG;
    ctx->fail_subbatch.store(index);
    return RSG_OK;
}

int rsg_set_tuning(const char* name, const char* value) {
    return rsg::set_tuning(name, value) ? RSG_ERR_INVALID_ARG : RSG_OK;
}

int rsg_get_tuning(const char* name, char* out, size_t cap) {
    return rsg::get_tuning(name, out, cap) ? RSG_ERR_INVALID_ARG : RSG_OK;
}

int rsg_set_record_engine(rsg_ctx* ctx, int engine) {
    int st = enter(ctx);
    if (st) return st;
    if (engine < RSG_RECORD_ENGINE_AUTO || engine > RSG_RECORD_ENGINE_TWO_PASS) return RSG_ERR_INVALID_ARG;
    ctx->record_engine.store(engine);
    return RSG_OK;
}

int rsg_last_kernel_ms(rsg_ctx* ctx, float* ms) {
    int st = enter(ctx);
    if (st) return st;
    if (!ms) return RSG_ERR_INVALID_ARG;
    *ms = ctx->last_kernel_ms.load();
    return RSG_OK;
}

// Heal (Erasure::heal, heal.rs:112-206) over n stripes of bitrot records.
int rsg_heal_records_submit(rsg_ctx* ctx, int k, int m, size_t shard_len, size_t n, const uint8_t* const* d_files,
                            uint8_t* const* d_targets, int algo, int* h_status, void* stream, uint64_t* ticket) {
    int st = enter(ctx);
    if (st) return st;
    if (!ticket) return RSG_ERR_INVALID_ARG;
    *ticket = 0;
    if ((st = check_geometry(k, m))) return st;
    if (m == 0) return RSG_ERR_ZERO_PARITY_SHARDS;
    if (!d_files || !d_targets || (n && !h_status)) return RSG_ERR_INVALID_ARG;
    const uint64_t* key = hash_key(algo);
    if (!key) return RSG_ERR_INVALID_ARG;
    if (n == 0 || shard_len == 0) {
        for (size_t x = 0; x < n; ++x) h_status[x] = RSG_OK;
        *ticket = done_ticket(ctx);
        return RSG_OK;
    }
    const int t = k + m;
    const uint64_t rec = 32 + shard_len;
    // Targets are written in the same pass that reads the sources: a target
    // range overlapping any source (or another target) would be silent
    // corruption (e.g. rewriting a rotten shard file in place), so it is
    // rejected up front.
    const uint64_t span = n * rec;
    for (int i = 0; i < t; ++i) {
        if (!d_targets[i]) continue;
        for (int j = 0; j < t; ++j)
            if ((d_files[j] && spans_overlap(d_targets[i], span, d_files[j], span)) ||
                (j != i && d_targets[j] && spans_overlap(d_targets[i], span, d_targets[j], span)))
                return RSG_ERR_INVALID_ARG;
    }
    auto rj = std::make_shared<RecJob>();
    rj->ctx = ctx;
    rj->heal = true;
    rj->k = k;
    rj->m = m;
    rj->t = t;
    rj->S = shard_len;
    rj->n = n;
    rj->rec = rec;
    rj->key = key;
    rj->files.assign(d_files, d_files + t);
    rj->targets.assign(d_targets, d_targets + t);
    rj->h_status = h_status;
    rj->s = pick_stream(ctx, stream);
    rj->sc = ctx->take_scratch();
    return submit_record_job(ctx, std::move(rj), heal_begin, heal_finish, ticket);
}

int rsg_heal_records_dev(rsg_ctx* ctx, int k, int m, size_t shard_len, size_t n, const uint8_t* const* d_files,
                         uint8_t* const* d_targets, int algo, uint8_t* d_work, int* h_status, void* stream) {
    (void)d_work;  // unused since ABI 3
    uint64_t t = 0;
    int st = rsg_heal_records_submit(ctx, k, m, shard_len, n, d_files, d_targets, algo, h_status, stream, &t);
    return st ? st : rsg_wait(ctx, t);
}

// Whole-shard-file verification (bitrot_verify, bitrot.rs:616-655) of n files.
int rsg_bitrot_verify_dev(rsg_ctx* ctx, int algo, size_t n_files, const uint8_t* const* d_files,
                          const size_t* file_lens, size_t want_size, size_t part_size, size_t shard_size,
                          int* h_status, void* stream) {
    int st = enter(ctx);
    if (st) return st;
    if (ctx->timing.load()) ctx->last_kernel_ms.store(-1.f);  // a call that returns early was not timed
    if (n_files && (!d_files || !file_lens || !h_status)) return RSG_ERR_INVALID_ARG;
    const bool streaming = algo == RSG_HASH_HIGHWAY256S || algo == RSG_HASH_HIGHWAY256S_LEGACY;
    if (!streaming && algo != RSG_HASH_NONE) return RSG_ERR_UNSUPPORTED;
    if (shard_size == 0 && part_size > 0) return RSG_ERR_INVALID_ARG;
    const uint64_t hs = streaming ? 32 : 0;
    // bitrot_shard_file_size (bitrot.rs:593-601)
    const uint64_t expect =
        (streaming && part_size) ? (part_size + shard_size - 1) / shard_size * hs + part_size : part_size;
    if (want_size != expect) {
        for (size_t f = 0; f < n_files; ++f) h_status[f] = RSG_ERR_FILE_SIZE_MISMATCH;
        return RSG_OK;
    }
    for (size_t f = 0; f < n_files; ++f)
        if (!d_files[f] && file_lens[f]) return RSG_ERR_INVALID_ARG;
    const uint64_t* key = streaming ? hash_key(algo) : nullptr;
    const uint64_t full = part_size ? part_size / shard_size : 0, tail = part_size - full * shard_size;
    const uint64_t recs = full + (tail ? 1 : 0);  // records in a complete file
    const uint64_t rec = hs + shard_size;
    hipStream_t s = pick_stream(ctx, stream);
    struct Lease {  // the call's scratch, back to the pool on every return
        rsg_ctx* ctx;
        std::unique_ptr<RecScratch> sc;
        ~Lease() { ctx->give_scratch(std::move(sc)); }
    } lease{ctx, ctx->take_scratch()};
    RecScratch& sc = *lease.sc;
    if (streaming && recs && (st = sc.ensure((size_t)recs * n_files, (size_t)recs * n_files))) return st;
    // records wholly inside each file are verified on the GPU (flags per
    // record, [file][record]); full records of up to kMaxHashBases files per
    // launch, then the short last records likewise; a short file's complete
    // records alone in a launch of its own
    std::vector<uint64_t> avail(n_files, 0);
    std::vector<size_t> bulk_full, bulk_tail;
    for (size_t f = 0; f < n_files; ++f) {
        const uint64_t len = std::min<uint64_t>(file_lens[f], want_size);
        uint64_t a = std::min<uint64_t>(len / rec, full);
        if (a == full && tail && len - full * rec >= hs + tail) a = recs;
        avail[f] = a;
        if (!streaming || !a) continue;
        if ((st = hip_status(hipMemsetAsync(sc.d + (size_t)f * recs, 1, a, s)))) return st;
        if (a >= full && full) bulk_full.push_back(f);
        if (a > full) bulk_tail.push_back(f);
    }
    sc.tmark(s);  // the kernel-timing hook brackets every verify launch of the call
    for (size_t f = 0; f < n_files; ++f) {
        if (!streaming || !avail[f] || avail[f] >= full) continue;
        rsg::HashParams h;  // a short file: its complete records alone
        std::memset(&h, 0, sizeof(h));
        std::memcpy(h.key, key, sizeof(h.key));
        h.len = shard_size;
        h.n = avail[f];
        h.stripe_stride = rec;
        h.nbases = 1;
        h.per_base = avail[f];
        h.digest_off = -(int64_t)hs;
        h.base[0] = d_files[f] + hs;
        h.flag_base[0] = sc.d + (size_t)f * recs;
        if ((st = hip_status(rsg::launch_hh256(h, s)))) return st;
    }
    for (int pass = 0; pass < 2; ++pass) {
        const std::vector<size_t>& list = pass == 0 ? bulk_full : bulk_tail;
        for (size_t g0 = 0; g0 < list.size(); g0 += rsg::kMaxHashBases) {
            const size_t g1 = std::min(list.size(), g0 + (size_t)rsg::kMaxHashBases);
            rsg::HashParams h;
            std::memset(&h, 0, sizeof(h));
            std::memcpy(h.key, key, sizeof(h.key));
            h.len = pass == 0 ? shard_size : tail;
            h.per_base = pass == 0 ? full : 1;
            h.n = (g1 - g0) * h.per_base;
            h.stripe_stride = rec;
            h.nbases = (uint32_t)(g1 - g0);
            h.digest_off = -(int64_t)hs;
            for (size_t x = g0; x < g1; ++x) {
                const size_t f = list[x];
                h.base[x - g0] = d_files[f] + (pass == 0 ? 0 : full * rec) + hs;
                h.flag_base[x - g0] = sc.d + (size_t)f * recs + (pass == 0 ? 0 : full);
            }
            if ((st = hip_status(rsg::launch_hh256(h, s)))) return st;
        }
    }
    sc.tmark(s);
    std::vector<uint8_t> flags(streaming ? (size_t)recs * n_files : 0);
    if (!flags.empty()) {
        if ((st = flags_to_host(sc, sc.d, flags.size(), flags.data(), s))) return st;
    } else if ((st = hip_status(hipStreamSynchronize(s)))) {
        return st;
    }
    // the reference reads records in order: the first bad or missing one decides
    for (size_t f = 0; f < n_files; ++f) {
        int res = RSG_OK;
        for (uint64_t r = 0; r < avail[f] && streaming; ++r)
            if (!flags[(size_t)f * recs + r]) {
                res = RSG_ERR_BITROT_MISMATCH;
                break;
            }
        if (res == RSG_OK && file_lens[f] < want_size) res = RSG_ERR_UNEXPECTED_EOF;
        if (res == RSG_OK && file_lens[f] > want_size) res = RSG_ERR_TRAILING_DATA;
        h_status[f] = res;
    }
    if (sc.timing) ctx->last_kernel_ms.store(sc.tsum());  // the stream was synchronised above
    return RSG_OK;
}

// ---- host-buffer API ----

int rsg_encode(rsg_ctx* ctx, int k, int m, size_t shard_len, uint8_t* const* shards) {
    int st = enter(ctx);
    if (st) return st;
    if ((st = check_geometry(k, m))) return st;
    if (m == 0) return RSG_ERR_ZERO_PARITY_SHARDS;
    if (!shards) return RSG_ERR_INVALID_ARG;
    for (int i = 0; i < k + m; ++i)
        if (!shards[i]) return RSG_ERR_INVALID_ARG;
    if (shard_len == 0) return RSG_ERR_EMPTY_SHARD;
    auto cd = get_codec(k, m);
    if (!cd) return RSG_ERR_INVALID_ARG;
    HostLane* lane;
    auto g = acquire_lane(ctx, lane);
    // one block per call: data in, parity out, the kernels read the device
    // copy at pitch S (back-to-back shards) or 256-aligned slots
    const bool in_one = contiguous(shards, 0, k, shard_len), out_one = contiguous(shards, k, m, shard_len);
    if (in_one && out_one && shards[k] == shards[0] + (size_t)k * shard_len && zero_copy_enabled()) {
        // a whole block in pinned memory: the kernels read the data and write
        // the parity over PCIe in place, no staging copies (per-block calls)
        if (uint8_t* dv = pinned_view(shards[0], (size_t)(k + m) * shard_len, ctx->device)) {
            if ((st = lane->ensure(0))) return st;
            RowSet rs = encode_rows(*cd, shard_len);
            if ((st = apply_rows(rs, dv, dv, 0, 0, shard_len, 1, rsg::GF_MODE_STORE, nullptr, lane->stream))) return st;
            return hip_status(hipStreamSynchronize(lane->stream));
        }
    }
    const uint64_t pitch = in_one ? shard_len : round_up(shard_len, 256);
    if ((st = lane->ensure((size_t)pitch * (k + m)))) return st;
    hipStream_t s = lane->stream;
    uint8_t* d = lane->d_buf;
    if (in_one) {
        if ((st = hip_status(hipMemcpyAsync(d, shards[0], (size_t)k * shard_len, hipMemcpyHostToDevice, s)))) return st;
    } else {
        for (int i = 0; i < k; ++i)
            if ((st = hip_status(hipMemcpyAsync(d + i * pitch, shards[i], shard_len, hipMemcpyHostToDevice, s))))
                return st;
    }
    RowSet rs = encode_rows(*cd, pitch);
    if ((st = apply_rows(rs, d, d, 0, 0, shard_len, 1, rsg::GF_MODE_STORE, nullptr, s))) return st;
    if (out_one && pitch == shard_len) {
        if ((st = hip_status(hipMemcpyAsync(shards[k], d + (size_t)k * pitch, (size_t)m * shard_len,
                                            hipMemcpyDeviceToHost, s))))
            return st;
    } else {
        for (int p = 0; p < m; ++p)
            if ((st = hip_status(hipMemcpyAsync(shards[k + p], d + (k + p) * pitch, shard_len, hipMemcpyDeviceToHost,
                                                s))))
                return st;
    }
    return hip_status(hipStreamSynchronize(s));
}

int rsg_reconstruct(rsg_ctx* ctx, int k, int m, size_t shard_len, uint8_t* const* shards, const uint8_t* present,
                    int mode) {
    int st = enter(ctx);
    if (st) return st;
    if ((st = check_geometry(k, m))) return st;
    if (!present || (shard_len && !shards)) return RSG_ERR_INVALID_ARG;
    if (mode < RSG_RECONSTRUCT_DATA || mode > RSG_RECONSTRUCT_REENCODE_PARITY) return RSG_ERR_INVALID_ARG;
    int npresent = 0;
    for (int i = 0; i < k + m; ++i) npresent += present[i] ? 1 : 0;
    if (shard_len == 0) {
        // recover_empty_payload_data_shards: erasure.rs:563-594 (any present shard
        // suffices) and bridge.rs:54-84 (reconstruct_opt path: needs k present).
        if (mode == RSG_RECONSTRUCT_MISSING) return npresent >= k ? RSG_OK : RSG_ERR_TOO_FEW_SHARDS;
        return npresent >= 1 ? RSG_OK : RSG_ERR_TOO_FEW_SHARDS;
    }
    if (npresent < k) return RSG_ERR_TOO_FEW_SHARDS;
    if (m == 0) return RSG_OK;
    if (npresent == k + m && mode != RSG_RECONSTRUCT_REENCODE_PARITY) return RSG_OK;
    for (int i = 0; i < k + m; ++i)
        if (!shards[i]) return RSG_ERR_INVALID_ARG;
    auto cd = get_codec(k, m);
    if (!cd) return RSG_ERR_INVALID_ARG;
    auto plan = cd->plan(present);
    if (!plan) return RSG_ERR_TOO_FEW_SHARDS;
    RowSet rs = reconstruct_rows(*cd, *plan, present, mode, 0);
    if (rs.R == 0) return RSG_OK;
    const std::vector<int> targets = reconstruct_targets(*cd, *plan, present, mode);
    HostLane* lane;
    auto g = acquire_lane(ctx, lane);
    const uint64_t pitch = round_up(shard_len, 256);
    if ((st = lane->ensure((size_t)pitch * (k + targets.size())))) return st;
    hipStream_t s = lane->stream;
    uint8_t* d = lane->d_buf;
    rs.in_off.clear();
    rs.out_off.clear();
    // Survivors go to slots 0..k-1 of the lane buffer, outputs to slots k.. .
    for (int c = 0; c < k; ++c) {
        if ((st = hip_status(hipMemcpyAsync(d + c * pitch, shards[plan->survivors[c]], shard_len,
                                            hipMemcpyHostToDevice, s))))
            return st;
        rs.in_off.push_back((uint64_t)c * pitch);
    }
    for (size_t r = 0; r < targets.size(); ++r) rs.out_off.push_back((uint64_t)(k + r) * pitch);
    if ((st = apply_rows(rs, d, d, 0, 0, shard_len, 1, rsg::GF_MODE_STORE, nullptr, s))) return st;
    for (size_t r = 0; r < targets.size(); ++r)
        if ((st = hip_status(hipMemcpyAsync(shards[targets[r]], d + (k + r) * pitch, shard_len,
                                            hipMemcpyDeviceToHost, s))))
            return st;
    return hip_status(hipStreamSynchronize(s));
}

int rsg_verify(rsg_ctx* ctx, int k, int m, size_t shard_len, const uint8_t* const* shards, int* ok) {
    int st = enter(ctx);
    if (st) return st;
    if ((st = check_geometry(k, m))) return st;
    if (!shards || !ok) return RSG_ERR_INVALID_ARG;
    *ok = 0;
    if (m == 0 || shard_len == 0) {
        *ok = 1;
        return RSG_OK;
    }
    for (int i = 0; i < k + m; ++i)
        if (!shards[i]) return RSG_ERR_INVALID_ARG;
    auto cd = get_codec(k, m);
    if (!cd) return RSG_ERR_INVALID_ARG;
    HostLane* lane;
    auto g = acquire_lane(ctx, lane);
    const uint64_t pitch = round_up(shard_len, 256);
    const uint64_t flag_off = pitch * (uint64_t)(2 * m + k);
    if ((st = lane->ensure((size_t)flag_off + 256))) return st;
    hipStream_t s = lane->stream;
    uint8_t* d = lane->d_buf;
    for (int i = 0; i < k + m; ++i)
        if ((st = hip_status(hipMemcpyAsync(d + i * pitch, shards[i], shard_len, hipMemcpyHostToDevice, s)))) return st;
    RowSet rs = encode_rows(*cd, pitch);
    uint8_t* d_flag = d + flag_off;
    if ((st = hip_status(hipMemsetAsync(d_flag, 1, 1, s)))) return st;
    if (k <= rsg::kMaxC) {
        // re-encode and compare in one pass (erasure.rs:430-441)
        if ((st = apply_rows(rs, d, d, 0, 0, shard_len, 1, rsg::GF_MODE_COMPARE, d_flag, s))) return st;
    } else {
        // k > 16 cannot compare inside a chained (GF_MODE_XOR) product: re-encode
        // into spare slots, then compare them with the given parity on the
        // device (identity rows in compare mode, <= 16 per launch)
        for (int p = 0; p < m; ++p) rs.out_off[p] = (uint64_t)(k + m + p) * pitch;
        if ((st = apply_rows(rs, d, d, 0, 0, shard_len, 1, rsg::GF_MODE_STORE, nullptr, s))) return st;
        for (int p0 = 0; p0 < m; p0 += rsg::kMaxC) {
            RowSet id;
            id.R = id.C = std::min(rsg::kMaxC, m - p0);
            id.coef.assign((size_t)id.R * id.C, 0);
            for (int i = 0; i < id.R; ++i) {
                id.coef[(size_t)i * id.C + i] = 1;
                id.in_off.push_back((uint64_t)(k + m + p0 + i) * pitch);
                id.out_off.push_back((uint64_t)(k + p0 + i) * pitch);
            }
            if ((st = apply_rows(id, d, d, 0, 0, shard_len, 1, rsg::GF_MODE_COMPARE, d_flag, s))) return st;
        }
    }
    uint8_t h = 0;
    if ((st = hip_status(hipMemcpyAsync(&h, d_flag, 1, hipMemcpyDeviceToHost, s)))) return st;
    if ((st = hip_status(hipStreamSynchronize(s)))) return st;
    *ok = h ? 1 : 0;
    return RSG_OK;
}

int rsg_hash(rsg_ctx* ctx, int algo, const uint8_t* data, size_t len, uint8_t out[32]) {
    int st = enter(ctx);
    if (st) return st;
    if (!out || (len && !data) || !hash_key(algo)) return RSG_ERR_INVALID_ARG;
    HostLane* lane;
    auto g = acquire_lane(ctx, lane);
    const uint64_t data_bytes = round_up(len ? len : 1, 256);
    if ((st = lane->ensure((size_t)data_bytes + 256))) return st;
    hipStream_t s = lane->stream;
    uint8_t* d = lane->d_buf;
    if (len && (st = hip_status(hipMemcpyAsync(d, data, len, hipMemcpyHostToDevice, s)))) return st;
    if ((st = hash_messages(algo, d, len, 1, 1, 0, 0, d + data_bytes, s))) return st;
    if ((st = hip_status(hipMemcpyAsync(out, d + data_bytes, 32, hipMemcpyDeviceToHost, s)))) return st;
    return hip_status(hipStreamSynchronize(s));
}

}  // extern "C"
