// scl_kernels.hip -- gfx950 kernels of the polar SC/SCL engine.
//
// Replaces the reference's frame loop (dl_scl_polar/eval/run_fer_sweep.py:79-121) and its
// list decoder (dl_scl_polar/polar/scl.py:108-209) with:
//
//   scl_decode_kernel  one 64-lane wavefront per codeword.  Lane i < L owns list path i
//                      (metric, rank, decided bits u, candidate bits, CRC syndrome, and a
//                      table of which LDS slot holds each depth of its LLR tree).  f/g
//                      node updates spread (path, element) pairs over all 64 lanes; the
//                      per-phase list update (metric, stable 2L->L selection) runs on the
//                      path lanes with cross-lane reads; the CRC-24 check is an incremental
//                      GF(2) syndrome.  The LLR tree never moves: a path forking only copies
//                      its slot table (lazy copy), because every live path rewrites the
//                      same depths at the same phase (successive cancellation is lockstep).
//   channel_kernel     the TX chain of run_fer_sweep.py:79-87 (payload, CRC attach, polar
//                      transform, BPSK, AWGN, LLR) from a counter-based Philox stream.
//
// Numerics follow the reference bit for bit: fp64 LLRs, exact min-sum f and g
// (polar.py:122-127), metric += np.logaddexp(0, +-llr) via a bit-exact port of glibc's
// exp/log1p (glibc_softplus.h), and Python's stable sort realised as a rank count on the
// key (metric, previous list position).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "glibc_softplus.h"
#include "scl_kernels.h"

namespace {

constexpr int kWave = 64;

__device__ __forceinline__ uint32_t bperm32(uint32_t v, int src) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)v);
}
__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src) {
    uint32_t lo = bperm32((uint32_t)v, src), hi = bperm32((uint32_t)(v >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ double shfl_f64(double v, int src) {
    return pscl_asf64(shfl_u64(pscl_asu64(v), src));
}
__device__ __forceinline__ uint32_t rdl_u32(uint32_t v, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ double rdl_f64(double v, int l) {
    uint64_t u = pscl_asu64(v);
    uint32_t lo = rdl_u32((uint32_t)u, l), hi = rdl_u32((uint32_t)(u >> 32), l);
    return pscl_asf64(((uint64_t)hi << 32) | lo);
}

// Orders the wave's LDS traffic: hardware executes one wave's LDS instructions in order;
// this keeps the compiler from moving loads above the stores they depend on.
__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// f(a,b) = sign(a) sign(b) min(|a|,|b|)  (polar.py:122-123; exact, sign(0)=0 gives +-0)
__device__ __forceinline__ double f_minsum(double a, double b) {
    double m = fmin(fabs(a), fabs(b));
    return ((a < 0.0) != (b < 0.0)) ? -m : m;
}
// g(a,b,c) = b + (1-2c) a  (polar.py:126-127; one rounding)
__device__ __forceinline__ double g_node(double a, double b, uint32_t c) { return c ? b - a : b + a; }

// Arikan transform of the low w bits of x (in-word, w <= 64): bit j ^= bit j+s for bit s of j
// clear, for every stage s (stages commute).  Bits >= w must be zero.
__device__ __forceinline__ uint64_t polar_transform64(uint64_t x) {
    x ^= (x >> 1) & 0x5555555555555555ULL;
    x ^= (x >> 2) & 0x3333333333333333ULL;
    x ^= (x >> 4) & 0x0f0f0f0f0f0f0f0fULL;
    x ^= (x >> 8) & 0x00ff00ff00ff00ffULL;
    x ^= (x >> 16) & 0x0000ffff0000ffffULL;
    x ^= (x >> 32) & 0x00000000ffffffffULL;
    return x;
}

__device__ __forceinline__ uint64_t pick_word(uint64_t w0, uint64_t w1, int idx) { return idx ? w1 : w0; }

// slot table: 5 bits per depth d in [1, n-1] at bit offset 5*d
__device__ __forceinline__ int slot_of(uint64_t tab, int d) { return (int)((tab >> (5 * d)) & 31u); }

template <int LMAX, bool HIST>
__global__ void __launch_bounds__(PSCL_MAX_WAVES_PER_WG * kWave)
    scl_decode_kernel(const pscl_decode_params P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t* T = reinterpret_cast<uint64_t*>(smem);  // exp table, 2 KB, shared by the WG
    for (int i = threadIdx.x; i < PSCL_EXP_TABLE_WORDS; i += blockDim.x) T[i] = P.exp_table[i];
    __syncthreads();

    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    unsigned char* wbase = smem + PSCL_EXP_TABLE_WORDS * 8 + (size_t)wave * P.wave_bytes;
    double* A = reinterpret_cast<double*>(wbase);                          // L*(N-2) LLRs
    uint8_t* inv = wbase + P.a_bytes;                                       // 64 B selection map
    double* hist_llr = reinterpret_cast<double*>(wbase + P.a_bytes + 64);   // [K][L]
    uint8_t* hist_par = wbase + P.a_bytes + 64 + (size_t)P.K * P.L * 8;     // [K][L]

    const int N = P.N, n = P.n, K = P.K, L = P.L, W = P.W;
    const int wpg = (int)(blockDim.x >> 6);
    const int64_t stride = (int64_t)gridDim.x * wpg;

    for (int64_t f = (int64_t)blockIdx.x * wpg + wave; f < P.B; f += stride) {
        const double* ch = P.llr + f * N;
        uint64_t fm0 = 0, fm1 = 0, fv0 = 0, fv1 = 0;
        if (P.force) {
            const uint64_t* fr = P.force + f * 2 * W;
            fm0 = fr[0];
            fv0 = fr[W];
            if (W > 1) {
                fm1 = fr[1];
                fv1 = fr[W + 1];
            }
        }
        // per-path state (meaningful in lanes < cnt)
        double metric = 0.0;
        int rank = 0;
        uint64_t u0 = 0, u1 = 0;    // decided bits u[phase]
        uint64_t ib0 = 0, ib1 = 0;  // candidate bits in info order
        uint32_t syn = 0;           // CRC syndrome of the candidate bits
        uint64_t tab = 0;           // LDS slot per depth
        int cnt = 1;                // live paths (wave-uniform)
        int j = 0;                  // info index (wave-uniform)

        for (int phi = 0; phi < N; ++phi) {
            const int t = phi ? __builtin_ctz(phi) : n;
            const int start = phi ? n - t : 1;
            // partial sums of the left sibling of the g node: transform of u[phi-w, phi)
            uint64_t xs = 0;
            if (phi) {
                const int w = 1 << t;
                const int lo = phi - w;
                uint64_t word = pick_word(u0, u1, lo >> 6);
                uint64_t seg = (w == 64) ? word : (word >> (lo & 63)) & ((1ULL << w) - 1);
                xs = polar_transform64(seg);
            }
            // ---- LLR tree: depths start .. n-1 into LDS slot = lane of the path
            for (int d = start; d < n; ++d) {
                const int lw = n - d, w = 1 << lw;
                const bool is_g = (d == start) && phi;
                const int total = cnt << lw;
                const int off_out = L * (N - 2 * w);
                const int off_in = L * (N - 4 * w);
                for (int base = 0; base < total; base += kWave) {
                    const int tt = base + lane;
                    const int i = tt >> lw;
                    const int e = tt & (w - 1);
                    const int isrc = i < kWave ? i : 0;
                    const uint64_t ti = shfl_u64(tab, isrc);
                    const uint64_t xi = is_g ? shfl_u64(xs, isrc) : 0;
                    if (tt < total) {
                        // the first step reads the parent through the path's slot table; deeper
                        // steps read the depth this phase just wrote into the path's own slot
                        const int ps = (d == start) ? slot_of(ti, d - 1) : i;
                        const double* par = (d == 1) ? ch : A + off_in + ps * (2 * w);
                        const double a = par[e], b = par[e + w];
                        A[off_out + i * w + e] = is_g ? g_node(a, b, (uint32_t)(xi >> e) & 1u) : f_minsum(a, b);
                    }
                }
                wave_lds_fence();
            }
            if (start < n) {
                uint64_t mask = 0, val = 0;
                for (int d = start; d < n; ++d) {
                    mask |= 31ULL << (5 * d);
                    val |= (uint64_t)lane << (5 * d);
                }
                tab = (tab & ~mask) | val;
            }
            // ---- leaf LLR of each path
            double lam = 0.0;
            if (lane < cnt) {
                const double* par = (n == 1) ? ch : A + L * (N - 4) + slot_of(tab, n - 1) * 2;
                const double a = par[0], b = par[1];
                lam = (phi & 1) ? g_node(a, b, (uint32_t)xs & 1u) : f_minsum(a, b);
            }
            // ---- path metric increments (scl.py:102-105), shared log1p(exp(-|llr|))
            const double Lt = pscl_softplus_tail(lam, T);
            const double m0 = metric + pscl_logaddexp0(-lam, Lt);
            const double m1 = metric + pscl_logaddexp0(lam, Lt);
            const uint64_t infow = pick_word(P.info_mask[0], P.info_mask[1], phi >> 6);
            const bool is_info = (infow >> (phi & 63)) & 1;
            const uint64_t fmw = pick_word(fm0, fm1, j >> 6), fvw = pick_word(fv0, fv1, j >> 6);
            // SC mode (sc_decode polar.py:149-153): every info bit is a hard decision llr < 0
            const bool forced = is_info && (P.sc_hard || ((fmw >> (j & 63)) & 1));

            if (!is_info || forced) {
                // single child per path; stable re-sort (scl.py:173) = rank on (metric, rank)
                uint32_t v = 0;
                if (forced) v = P.sc_hard ? (uint32_t)(lam < 0.0) : (uint32_t)(fvw >> (j & 63)) & 1u;
                metric = v ? m1 : m0;
                if (v) {
                    if (phi < 64) u0 |= 1ULL << phi; else u1 |= 1ULL << (phi - 64);
                    if (j < 64) ib0 |= 1ULL << j; else ib1 |= 1ULL << (j - 64);
                    syn ^= P.crc_cols[j];
                }
                if (HIST && is_info && lane < cnt) {
                    hist_llr[j * L + lane] = lam;
                    hist_par[j * L + lane] = (uint8_t)lane;
                }
                if (cnt > 1) {
                    int r = 0;
#pragma unroll
                    for (int k = 0; k < LMAX; ++k) {
                        if (k < cnt) {
                            const double mk = rdl_f64(metric, k);
                            const int rk = (int)rdl_u32((uint32_t)rank, k);
                            r += (mk < metric) || (mk == metric && rk < rank);
                        }
                    }
                    rank = r;
                }
            } else {
                // free info bit: children (bit0, bit1) of each path in list order,
                // stable sort on (metric, 2*rank + bit), keep the first L (scl.py:163-174)
                int r0 = 0, r1 = 0;
                const int k0 = 2 * rank, k1 = 2 * rank + 1;
#pragma unroll
                for (int k = 0; k < LMAX; ++k) {
                    if (k < cnt) {
                        const double a0 = rdl_f64(m0, k), a1 = rdl_f64(m1, k);
                        const int kk = 2 * (int)rdl_u32((uint32_t)rank, k);
                        r0 += (a0 < m0) || (a0 == m0 && kk < k0);
                        r0 += (a1 < m0) || (a1 == m0 && kk + 1 < k0);
                        r1 += (a0 < m1) || (a0 == m1 && kk < k1);
                        r1 += (a1 < m1) || (a1 == m1 && kk + 1 < k1);
                    }
                }
                const int ncnt = (2 * cnt < L) ? 2 * cnt : L;
                if (lane < cnt) {
                    if (r0 < ncnt) inv[r0] = (uint8_t)(2 * lane);
                    if (r1 < ncnt) inv[r1] = (uint8_t)(2 * lane + 1);
                }
                wave_lds_fence();
                const int sel = (lane < ncnt) ? inv[lane] : 0;
                const int p = sel >> 1;
                const uint32_t b = (uint32_t)sel & 1u;
                const double pm0 = shfl_f64(m0, p), pm1 = shfl_f64(m1, p);
                const double plam = shfl_f64(lam, p);
                const uint64_t pu0 = shfl_u64(u0, p), pu1 = shfl_u64(u1, p);
                const uint64_t pib0 = shfl_u64(ib0, p), pib1 = shfl_u64(ib1, p);
                const uint64_t ptab = shfl_u64(tab, p);
                const uint32_t psyn = bperm32(syn, p);
                wave_lds_fence();  // inv[] is rewritten at the next free phase
                metric = b ? pm1 : pm0;
                u0 = pu0;
                u1 = pu1;
                ib0 = pib0;
                ib1 = pib1;
                tab = ptab;
                syn = psyn;
                if (b) {
                    if (phi < 64) u0 |= 1ULL << phi; else u1 |= 1ULL << (phi - 64);
                    if (j < 64) ib0 |= 1ULL << j; else ib1 |= 1ULL << (j - 64);
                    syn ^= P.crc_cols[j];
                }
                rank = lane;
                cnt = ncnt;
                if (HIST && lane < cnt) {
                    hist_llr[j * L + lane] = plam;
                    hist_par[j * L + lane] = (uint8_t)p;
                }
            }
            if (is_info) ++j;
        }

        // ---- epilogue: list in rank order, best = first CRC-passing candidate (scl.py:190-201)
        const bool active = lane < cnt;
        const bool pass = active && P.has_crc && syn == 0;
        int best_rank = 0;
        if (P.has_crc) {
            int cand = pass ? rank : 1 << 20;
#pragma unroll
            for (int k = 0; k < LMAX; ++k)
                if (k < cnt) {
                    const int ck = (int)rdl_u32((uint32_t)cand, k);
                    best_rank = (k == 0 || ck < best_rank) ? ck : best_rank;
                }
            if (best_rank >= (1 << 20)) best_rank = 0;
        }
        if (active) {
            const int64_t row = f * L + rank;
            if (P.metrics) P.metrics[row] = metric;
            if (P.cands) {
                P.cands[row * W] = ib0;
                if (W > 1) P.cands[row * W + 1] = ib1;
            }
            if (HIST && P.info_llrs) {
                int cur = lane;
                for (int jj = K - 1; jj >= 0; --jj) {
                    P.info_llrs[row * K + jj] = hist_llr[jj * L + cur];
                    cur = hist_par[jj * L + cur];
                }
            }
            if (rank == best_rank) {
                const bool bpass = P.has_crc ? (syn == 0) : true;
                if (P.best) {
                    P.best[f * W] = ib0;
                    if (W > 1) P.best[f * W + 1] = ib1;
                }
                if (P.flags) P.flags[f] = (uint8_t)((bpass ? PSCL_FLAG_CRC_PASS : 0u) | (uint32_t)best_rank);
                if (P.n_paths) P.n_paths[f] = cnt;
                if (P.ref) {
                    const uint64_t r0 = P.ref[f * W], r1 = (W > 1) ? P.ref[f * W + 1] : 0;
                    const uint64_t d0 = ib0 ^ r0, d1 = ib1 ^ r1;
                    const int bit_err = __popcll(d0) + __popcll(d1);
                    const int kp = P.k_payload;
                    const uint64_t pm0 = kp >= 64 ? ~0ULL : ((1ULL << kp) - 1);
                    const uint64_t pm1 = kp >= 128 ? ~0ULL : (kp > 64 ? ((1ULL << (kp - 64)) - 1) : 0ULL);
                    const int pay_err = __popcll(d0 & pm0) + __popcll(d1 & pm1);
                    unsigned long long* C = reinterpret_cast<unsigned long long*>(P.counters);
                    if (!bpass) atomicAdd(C + PSCL_CNT_FRAME_ERR, 1ULL);
                    if (bit_err) atomicAdd(C + PSCL_CNT_BIT_ERR, (unsigned long long)bit_err);
                    if (pay_err) {
                        atomicAdd(C + PSCL_CNT_PAYLOAD_ERR, 1ULL);
                        atomicAdd(C + PSCL_CNT_PAYLOAD_BIT, (unsigned long long)pay_err);
                    }
                }
            }
        }
        // next frame reuses A/inv/hist: keep this frame's LDS reads ahead of its writes
        wave_lds_fence();
    }
    if (P.ref && blockIdx.x == 0 && threadIdx.x == 0)
        atomicAdd(reinterpret_cast<unsigned long long*>(P.counters) + PSCL_CNT_FRAMES, (unsigned long long)P.B);
}

// ------------------------------------------------------------------------ channel (TX)

struct u32x4 {
    uint32_t x, y, z, w;
};

// Philox4x32-10 (Salmon et al., SC'11)
__device__ __forceinline__ u32x4 philox4x32(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
        c = u32x4{(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1, (uint32_t)p0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

__global__ void __launch_bounds__(256) channel_kernel(const pscl_channel_params P) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t stride = (int64_t)gridDim.x * 4;
    const uint32_t k0 = (uint32_t)P.seed, k1 = (uint32_t)(P.seed >> 32) ^ (P.stream_id * 0x85EBCA6Bu);
    for (int64_t idx = (int64_t)blockIdx.x * 4 + wave; idx < P.B; idx += stride) {
        const uint64_t fr = (uint64_t)(P.frame0 + idx);
        // payload: k_payload uniform bits from one Philox block (draw id 0xffffffff)
        const u32x4 rb = philox4x32(u32x4{(uint32_t)fr, (uint32_t)(fr >> 32), 0xffffffffu, 0u}, k0, k1);
        const uint64_t r0 = ((uint64_t)rb.y << 32) | rb.x, r1 = ((uint64_t)rb.w << 32) | rb.z;
        const int kp = P.k_payload;
        uint64_t m0 = kp >= 64 ? r0 : (r0 & ((1ULL << kp) - 1));
        uint64_t m1 = kp > 64 ? (r1 & ((kp >= 128) ? ~0ULL : ((1ULL << (kp - 64)) - 1))) : 0;
        // CRC remainder (attach_crc crc.py:19-37) as XOR of per-payload-bit columns
        uint32_t rem = 0;
        for (int q = 0; q < kp; ++q) {
            const uint64_t wq = q < 64 ? m0 : m1;
            if ((wq >> (q & 63)) & 1) rem ^= P.attach_cols[q];
        }
        for (int i = 0; i < P.crc_deg; ++i) {
            const int q = kp + i;
            if ((rem >> i) & 1) {
                if (q < 64) m0 |= 1ULL << q; else m1 |= 1ULL << (q - 64);
            }
        }
        // u[info_set[q]] = msg[q]; x = polar transform of u (polar.py:17-29,106-119)
        uint64_t x0 = 0, x1 = 0;
        for (int q = 0; q < P.K; ++q) {
            const uint64_t wq = q < 64 ? m0 : m1;
            if ((wq >> (q & 63)) & 1) {
                const int pos = P.info_set[q];
                if (pos < 64) x0 |= 1ULL << pos; else x1 |= 1ULL << (pos - 64);
            }
        }
        x0 = polar_transform64(x0);
        x1 = polar_transform64(x1);
        if (P.N > 64) x0 ^= x1;  // stage step 64
        if (P.msg && lane == 0) {
            P.msg[idx * P.W] = m0;
            if (P.W > 1) P.msg[idx * P.W + 1] = m1;
        }
        // AWGN: lane handles positions lane and lane+64 with one Box-Muller pair
        const u32x4 rn = philox4x32(u32x4{(uint32_t)fr, (uint32_t)(fr >> 32), (uint32_t)lane, 0u}, k0, k1);
        const uint64_t a = ((uint64_t)rn.y << 32) | rn.x, bb = ((uint64_t)rn.w << 32) | rn.z;
        const double uu1 = ((double)(a >> 11) + 1.0) * 0x1p-53;  // (0, 1]
        const double uu2 = (double)(bb >> 11) * 0x1p-53;         // [0, 1)
        const double rad = sqrt(-2.0 * log(uu1));
        double sn, cs;
        sincospi(2.0 * uu2, &sn, &cs);
        const double z[2] = {rad * cs, rad * sn};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int pos = lane + 64 * h;
            if (pos < P.N) {
                const uint64_t xw = pos < 64 ? x0 : x1;
                const double sym = ((xw >> (pos & 63)) & 1) ? -1.0 : 1.0;
                const double received = sym + P.sigma * z[h];
                P.llr[idx * P.N + pos] = 2.0 * received / P.noise_var;
            }
        }
    }
}

}  // namespace

// ------------------------------------------------------------------------- launchers

// waves (frames) per workgroup: as many as fit 160 KB of LDS, at most PSCL_MAX_WAVES_PER_WG
int pscl_decode_wpg(const pscl_decode_params& P) {
    const int avail = 160 * 1024 - PSCL_EXP_TABLE_WORDS * 8;
    int w = avail / (P.wave_bytes > 0 ? P.wave_bytes : 1);
    return w > PSCL_MAX_WAVES_PER_WG ? PSCL_MAX_WAVES_PER_WG : w;
}

static int decode_lds_bytes(const pscl_decode_params& P, int hist) {
    (void)hist;
    return PSCL_EXP_TABLE_WORDS * 8 + pscl_decode_wpg(P) * P.wave_bytes;
}

template <int LMAX>
static hipError_t launch_l(const pscl_decode_params& P, int hist, int64_t grid, hipStream_t s) {
    const int lds = decode_lds_bytes(P, hist);
    const int threads = pscl_decode_wpg(P) * kWave;
    if (hist) {
        hipLaunchKernelGGL((scl_decode_kernel<LMAX, true>), dim3((unsigned)grid), dim3(threads), lds, s, P);
    } else {
        hipLaunchKernelGGL((scl_decode_kernel<LMAX, false>), dim3((unsigned)grid), dim3(threads), lds, s, P);
    }
    return hipGetLastError();
}

int pscl_decode_lmax(int L) {
    if (L <= 1) return 1;
    if (L <= 2) return 2;
    if (L <= 4) return 4;
    if (L <= 8) return 8;
    if (L <= 16) return 16;
    return 32;
}

int64_t pscl_decode_grid(const pscl_decode_params& P) {
    const int wpg = pscl_decode_wpg(P);
    int64_t g = (P.B + wpg - 1) / wpg;
    const int64_t cap = 1 << 20;
    return g < 1 ? 1 : (g > cap ? cap : g);
}

hipError_t pscl_launch_decode(const pscl_decode_params& P, int hist, hipStream_t s) {
    if (pscl_decode_wpg(P) < 1) return hipErrorInvalidValue;
    const int64_t grid = pscl_decode_grid(P);
    switch (pscl_decode_lmax(P.L)) {
        case 1: return launch_l<1>(P, hist, grid, s);
        case 2: return launch_l<2>(P, hist, grid, s);
        case 4: return launch_l<4>(P, hist, grid, s);
        case 8: return launch_l<8>(P, hist, grid, s);
        case 16: return launch_l<16>(P, hist, grid, s);
        default: return launch_l<32>(P, hist, grid, s);
    }
}

int pscl_decode_lds(const pscl_decode_params& P, int hist) { return decode_lds_bytes(P, hist); }

hipError_t pscl_launch_channel(const pscl_channel_params& P, hipStream_t s) {
    int64_t grid = (P.B + 3) / 4;
    if (grid > (1 << 20)) grid = 1 << 20;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(channel_kernel, dim3((unsigned)grid), dim3(256), 0, s, P);
    return hipGetLastError();
}
