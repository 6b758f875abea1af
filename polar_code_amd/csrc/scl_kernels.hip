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
#include <stdlib.h>

#include "glibc_softplus.h"
#include "scl_device.h"
#include "scl_kernels.h"

namespace {

using namespace pscl;

template <int LMAX, bool HIST>
__global__ void __launch_bounds__(PSCL_MAX_WAVES_PER_WG * kWave)
    scl_decode_kernel(const pscl_decode_params P) {
    constexpr int G = 2 * LMAX;      // lanes per frame
    constexpr int F = kWave / G;     // frames per wavefront
    constexpr int LOG_G = __builtin_ctz(G);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t* T = reinterpret_cast<uint64_t*>(smem);  // exp table, 2 KB, shared by the WG
    for (int i = threadIdx.x; i < PSCL_EXP_TABLE_WORDS; i += blockDim.x) T[i] = P.exp_table[i];
    __syncthreads();

    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int fl = lane >> LOG_G;        // frame slot of this lane
    const int g = lane & (G - 1);        // lane within the frame group
    const int gbase = lane & ~(G - 1);
    const int N = P.N, n = P.n, K = P.K, L = P.L, W = P.W;
    // per frame in LDS: the N channel LLRs, then L slots for each stored depth 2..n-1
    // (depth 1 is recomputed from the channel LLRs when depth 2 needs it)
    const int fstride = N + (N >= 8 ? L * (N / 2 - 2) : 0);
    const int half = N >> 1;
    unsigned char* wbase = smem + PSCL_EXP_TABLE_WORDS * 8 + (size_t)wave * P.wave_bytes;
    double* A = reinterpret_cast<double*>(wbase);                                     // [F][fstride]
    uint8_t* inv = wbase + P.a_bytes;                                                  // [64]
    double* hist_llr = reinterpret_cast<double*>(wbase + P.a_bytes + 64) + (size_t)fl * K * L;
    uint8_t* hist_par = wbase + P.a_bytes + 64 + (size_t)F * K * L * 8 + (size_t)fl * N * L;  // [N][L]
    double* Af = A + fl * fstride;       // this lane's frame

    const int wpg = (int)(blockDim.x >> 6);
    const int64_t wstride = (int64_t)gridDim.x * wpg * F;
    const bool path_lane = g < L;
    // candidate c = g: (path g, bit 0) for g < LMAX, (path g-LMAX, bit 1) for g >= LMAX
    const int cpath = g & (LMAX - 1);
    const uint32_t cbit = g >= LMAX ? 1u : 0u;

    // live batch size: P.B, or a device-side count bounded by P.B, or (DL-SCL retry rounds)
    // the total of the bucket lists (no warm start here: every frame decodes from phase 0)
    int bpre[PSCL_DL_NSEG + 1];
    int64_t Bn = P.d_count ? (*P.d_count < P.B ? (int64_t)*P.d_count : P.B) : P.B;
    if (P.elist) {
        const int64_t tot = pscl_bucket_prefix(P.bcount, P.bcap, bpre);
        Bn = tot < P.B ? tot : P.B;
    }
    for (int64_t f0 = ((int64_t)blockIdx.x * wpg + wave) * F; f0 < Bn; f0 += wstride) {
        const int64_t fi = f0 + fl;
        const bool fvalid = fi < Bn;
        const int64_t fsafe = fvalid ? fi : f0;
        // f indexes the force words and outputs: the frame index, or a bucket list's entry id
        const int64_t f = P.elist ? pscl_elist_entry(P, fsafe, bpre) : fi;
        const int64_t frow = P.fidx ? P.fidx[P.elist ? f : fsafe] : fsafe;
        // best / flags / counts at the frame's own row (the exact re-decode of screened frames) or at f
        const int64_t fo = P.out_by_row ? frow : f;
        if (P.rm_E == 0) {  // stage this frame's channel LLRs in LDS (read at every depth-1 use)
            const double* src = P.llr + frow * N;
            for (int x = g; x < N; x += G) Af[x] = src[x];
        } else {  // NR: de-rate-match + de-interleave while staging
            const double* src = P.llr + frow * P.rm_E;
            for (int x = g; x < N; x += G) Af[x] = nr_stage(src, P.rm_src[x], P.rm_E, N);
        }
        wave_lds_fence();
        const double* ch = Af;
        uint64_t fm0 = 0, fm1 = 0, fv0 = 0, fv1 = 0;
        if (P.force && fvalid) {
            const uint64_t* fr = P.force + f * 2 * W;
            fm0 = fr[0];
            fv0 = fr[W];
            if (W > 1) {
                fm1 = fr[1];
                fv1 = fr[W + 1];
            }
        }
        double metric = 0.0;
        uint64_t u0 = 0, u1 = 0;    // decided bits u[phase]
        uint32_t tab = 0;           // LDS slot per depth d (5 bits at 5*(d-1))
        int cnt = 1;                // live paths of this frame (group-uniform)
        int cu = 1;                 // wave-uniform bound: max live paths over the wave's frames
        int j = 0;                  // info index (wave-uniform)

        for (int phi = 0; phi < N; ++phi) {
            const int t = phi ? __builtin_ctz(phi) : n;
            const int start = phi ? n - t : 1;
            uint64_t xs = 0;  // partial sums of the left sibling of the g node
            if (phi) {
                const int w = 1 << t;
                const int lo = phi - w;
                const uint64_t word = pick_word(u0, u1, lo >> 6);
                const uint64_t seg = (w == 64) ? word : (word >> (lo & 63)) & ((1ULL << w) - 1);
                xs = polar_transform64(seg);
            }
            // ---- LLR tree, depths start .. n-1: element (frame fl2, path i, index e)
            const int lp = cu <= 1 ? 0 : 32 - __builtin_clz(cu - 1);  // log2 of pow2 >= cu
            const bool right1 = phi >= half;  // depth-1 node on the path: right child of the root
            // depth-1 value x of path data xp1 (transform of u[0, N/2)), recomputed from the channel
            auto d1 = [&](const double* chf, int x, uint64_t xp1) -> double {
                const double a = chf[x], b = chf[x + half];
                return right1 ? g_node(a, b, (uint32_t)(xp1 >> x) & 1u) : f_minsum(a, b);
            };
            uint64_t xp1 = 0;
            if (right1) xp1 = polar_transform64(half >= 64 ? u0 : (u0 & ((1ULL << half) - 1)));
            for (int d = (start > 2 ? start : 2); d < ((PSCL_ABLATE & 4) ? 0 : n); ++d) {
                const int lw = n - d, w = 1 << lw;
                const bool is_g = (d == start) && phi;
                const int total = F << (lp + lw);
                const int off_out = N + L * (half - 2 * w);
                const int off_in = N + L * (half - 4 * w);
                for (int base = 0; base < total; base += kWave) {
                    const int tt = base + lane;
                    const int fl2 = tt >> (lp + lw);
                    const int i = (tt >> lw) & ((1 << lp) - 1);
                    const int e = tt & (w - 1);
                    const int src = ((fl2 & (F - 1)) << LOG_G) | i;
                    uint32_t ti = 0;
                    uint64_t xi = 0, x1 = 0;
                    if (d == 2) {
                        if (right1) x1 = shfl_u64(xp1, src);
                    } else if (d == start) {
                        ti = bperm32(tab, src);
                    }
                    if (is_g) xi = shfl_u64(xs, src);
                    if (tt < total && i < cu) {
                        double* A2 = A + fl2 * fstride;
                        double a, b;
                        if (d == 2) {
                            a = d1(A2, e, x1);
                            b = d1(A2, e + w, x1);
                        } else {
                            const int ps = (d == start) ? (int)((ti >> (5 * (d - 3))) & 31u) : i;
                            const double* par = A2 + off_in + ps * (2 * w);
                            a = par[e];
                            b = par[e + w];
                        }
                        A2[off_out + i * w + e] = is_g ? g_node(a, b, (uint32_t)(xi >> e) & 1u) : f_minsum(a, b);
                    }
                }
                wave_lds_fence();
            }
            if (start < n && n > 2) {
                uint32_t mask = 0, val = 0;
                for (int d = (start > 2 ? start : 2); d < n; ++d) {
                    mask |= 31u << (5 * (d - 2));
                    val |= (uint32_t)g << (5 * (d - 2));
                }
                tab = (tab & ~mask) | val;
            }
            // ---- leaf LLR of each path (lanes g < L)
            double lam = 0.0;
            if (path_lane) {
                double a, b;
                if (n == 1) {
                    a = ch[0];
                    b = ch[1];
                } else if (n == 2) {
                    a = d1(ch, 0, xp1);
                    b = d1(ch, 1, xp1);
                } else {
                    const double* par = Af + N + L * (half - 4) + ((tab >> (5 * (n - 3))) & 31u) * 2;
                    a = par[0];
                    b = par[1];
                }
                lam = (phi & 1) ? g_node(a, b, (uint32_t)xs & 1u) : f_minsum(a, b);
            }
            // ---- metric increments (scl.py:102-105), shared log1p(exp(-|llr|))
            const double Lt = (PSCL_ABLATE & 1) ? lam * 0.5 : pscl_softplus_tail_bf(lam, T);
            const double m0 = metric + pscl_logaddexp0(-lam, Lt);
            const double m1 = metric + pscl_logaddexp0(lam, Lt);
            const uint64_t infow = pick_word(P.info_mask[0], P.info_mask[1], phi >> 6);
            const bool is_info = (infow >> (phi & 63)) & 1;
            // candidate key of this lane: (metric of child, 2 * list position + bit)
            const uint64_t m1b = pscl_asu64(m1);
            const uint64_t pm1 = ((uint64_t)from_lower_half<G, LMAX>((uint32_t)(m1b >> 32), lane) << 32) |
                                 from_lower_half<G, LMAX>((uint32_t)m1b, lane);
            uint64_t km = cbit ? pm1 : pscl_asu64(m0);
            bool kval = cpath < cnt;
            int ncnt = cnt;
            if (!is_info) {
                kval = kval && cbit == 0;  // frozen: bit 0 (scl.py:149-153)
            } else {
                const uint64_t fmw = pick_word(fm0, fm1, j >> 6), fvw = pick_word(fv0, fv1, j >> 6);
                if (P.sc_hard) {
                    const double plam = shfl_f64(lam, gbase + cpath);
                    kval = kval && cbit == (uint32_t)(plam < 0.0);  // sc_decode polar.py:149-153
                } else if ((fmw >> (j & 63)) & 1) {
                    kval = kval && cbit == (uint32_t)((fvw >> (j & 63)) & 1);  // forced (scl.py:146-161)
                } else {
                    ncnt = 2 * cnt < L ? 2 * cnt : L;  // both children (scl.py:163-168)
                }
            }
            if (!kval) km = 0x7ff0000000000000ULL;  // +inf: never ranks ahead of a live child
            const uint32_t kt = kval ? 2u * (uint32_t)cpath + cbit : 0x7fffffffu;
            // stable sort of the children, keep the first L (scl.py:173-174): rank count
            uint32_t r = 0;
            if (!(PSCL_ABLATE & 2)) rank_step<G, 1>((uint32_t)(km >> 32), (uint32_t)km, kt, lane, r);
            else r = kt;
            if (kval && r < (uint32_t)ncnt) inv[gbase + r] = (uint8_t)g;
            wave_lds_fence();
            const int c = (g < ncnt) ? inv[gbase + g] : g;
            const int par_g = c & (LMAX - 1);
            const uint32_t b = c >= LMAX ? 1u : 0u;
            const int ps2 = gbase + par_g;
            const uint64_t nm = shfl_u64(km, gbase + c);
            const uint64_t nu0 = shfl_u64(u0, ps2);
            const uint64_t nu1 = (N > 64) ? shfl_u64(u1, ps2) : 0;
            const uint32_t ntab = bperm32(tab, ps2);
            double nlam = 0.0;
            if (HIST) nlam = shfl_f64(lam, ps2);
            wave_lds_fence();  // inv[] is rewritten next phase
            metric = pscl_asf64(nm);
            u0 = nu0;
            u1 = nu1;
            tab = ntab;
            if (b) {
                if (phi < 64) u0 |= 1ULL << phi; else u1 |= 1ULL << (phi - 64);
            }
            if (HIST && g < ncnt) {
                if (is_info) hist_llr[j * L + g] = nlam;  // decision LLR (scl.py:158,166)
                hist_par[phi * L + g] = (uint8_t)par_g;   // list position before this phase
            }
            cnt = ncnt;
            if (is_info) {
                if (!P.sc_hard) cu = 2 * cu < L ? 2 * cu : L;
                ++j;
            }
        }

        // ---- epilogue: candidate bits u[info_set] and their CRC syndrome, rebuilt once from u
        uint64_t ib0 = 0, ib1 = 0;
        uint32_t syn = 0;
        for (int jj = 0; jj < K; ++jj) {
            const int ph = P.info_set[jj];
            const uint64_t bit = (pick_word(u0, u1, ph >> 6) >> (ph & 63)) & 1ULL;
            if (jj < 64) ib0 |= bit << jj; else ib1 |= bit << (jj - 64);
            syn ^= bit ? P.crc_cols[jj] : 0u;
        }
        // the list is in lane order; best = first CRC-passing candidate (scl.py:190-201)
        const bool active = path_lane && g < cnt && fvalid;
        const uint64_t passmask = __ballot(active && syn == 0);
        const uint64_t gmask = (passmask >> gbase) & ((G == 64) ? ~0ULL : ((1ULL << G) - 1));
        const int best = (P.has_crc && gmask) ? __builtin_ctzll(gmask) : 0;
        if (active) {
            const int64_t row = f * L + g;
            if (P.metrics) P.metrics[row] = metric;
            if (P.cands) {
                P.cands[row * W] = ib0;
                if (W > 1) P.cands[row * W + 1] = ib1;
            }
            if (HIST && P.info_llrs) {  // trace the path's history back through every phase
                int cur = g, jj = K - 1;
                for (int ph = N - 1; ph >= 0; --ph) {
                    if ((pick_word(P.info_mask[0], P.info_mask[1], ph >> 6) >> (ph & 63)) & 1) {
                        P.info_llrs[row * K + jj] = hist_llr[jj * L + cur];
                        --jj;
                    }
                    cur = hist_par[ph * L + cur];
                }
            }
            if (g == best) {
                const bool bpass = P.has_crc ? (syn == 0) : true;
                if (HIST && P.best_info_llrs) {
                    int cur = g, jj = K - 1;
                    for (int ph = N - 1; ph >= 0; --ph) {
                        if ((pick_word(P.info_mask[0], P.info_mask[1], ph >> 6) >> (ph & 63)) & 1) {
                            P.best_info_llrs[f * K + jj] = hist_llr[jj * L + cur];
                            --jj;
                        }
                        cur = hist_par[ph * L + cur];
                    }
                }
                if (P.best) {
                    P.best[fo * W] = ib0;
                    if (W > 1) P.best[fo * W + 1] = ib1;
                }
                if (P.flags) P.flags[fo] = (uint8_t)((bpass ? PSCL_FLAG_CRC_PASS : 0u) | (uint32_t)best);
                if (P.n_paths) P.n_paths[fo] = cnt;
                if (P.ref) {
                    const uint64_t r0 = P.ref[fo * W], r1 = (W > 1) ? P.ref[fo * W + 1] : 0;
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
        wave_lds_fence();  // the next frames reuse this wave's LDS
    }
    if (P.ref && !P.out_by_row && blockIdx.x == 0 && threadIdx.x == 0)  // (a re-decode's frames were counted)
        atomicAdd(reinterpret_cast<unsigned long long*>(P.counters) + PSCL_CNT_FRAMES, (unsigned long long)P.B);
}

// ------------------------------------------------------------------------ channel (TX)

// (u32x4, philox4x32, bm_pair: scl_device.h, shared with the fused-TX lane kernel)

// TX chain, two phases per wavefront of 64 frames:
//   A  lane = frame: Philox payload, CRC remainder and codeword from byte tables (both maps
//      are GF(2)-linear), message words stored;
//   B  per frame: its codeword broadcast through SGPRs, lanes generate the Box-Muller pairs
//      and store the LLR row with coalesced writes.
// Stream: payload = Philox(frame, draw 0xffffffff); noise pair c = lane + 64 q of a frame =
// Philox(frame, c) -> symbols c + 64 q and c + 64 q + 64 (c < 64).  With P.unc_counters the
// uncoded baseline of the same frames is counted in phase A too (the payload already drawn;
// noise pairs Philox(frame, 0x40000000 + c), as uncoded_kernel): one launch for the TX chain and
// the uncoded BPSK baseline of run_fer_sweep.py:79-121.
__global__ void __launch_bounds__(256) channel_kernel(const pscl_channel_params P) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t k0 = (uint32_t)P.seed, k1 = (uint32_t)(P.seed >> 32) ^ (P.stream_id * 0x85EBCA6Bu);
    const int E = P.rm_E ? P.rm_E : P.N;
    const int kp = P.k_payload;
    const int nb = (P.K + 7) >> 3, nbp = (kp + 7) >> 3;
    if (P.unc_counters && blockIdx.x == 0 && threadIdx.x == 0)
        atomicAdd(reinterpret_cast<unsigned long long*>(P.unc_counters) + PSCL_CNT_FRAMES, (unsigned long long)P.B);
    int ufe = 0, ube = 0;  // this lane's uncoded error counts (added once per workgroup at the end)
    for (int64_t base = ((int64_t)blockIdx.x * 4 + wave) * 64; base < P.B; base += (int64_t)gridDim.x * 256) {
        // ---- A: one frame per lane
        const int64_t idx = base + lane;
        const uint64_t fr = (uint64_t)(P.frame0 + idx);
        const u32x4 rb = philox4x32(u32x4{(uint32_t)fr, (uint32_t)(fr >> 32), 0xffffffffu, 0u}, k0, k1);
        const uint64_t r0 = ((uint64_t)rb.y << 32) | rb.x, r1 = ((uint64_t)rb.w << 32) | rb.z;
        uint64_t m0 = kp >= 64 ? r0 : (r0 & ((1ULL << kp) - 1));
        uint64_t m1 = kp > 64 ? (r1 & ((kp >= 128) ? ~0ULL : ((1ULL << (kp - 64)) - 1))) : 0;
        uint32_t rem = 0;  // attach_crc (crc.py:19-37)
        for (int k = 0; k < nbp; ++k)
            rem ^= P.crctab[k * 256 + (uint32_t)(((k < 8 ? m0 : m1) >> (8 * (k & 7))) & 255u)];
        if (P.crc_deg) {
            const uint64_t rw = (uint64_t)rem;
            if (kp < 64) {
                m0 |= rw << kp;
                if (kp + P.crc_deg > 64) m1 |= rw >> (64 - kp);
            } else {
                m1 |= rw << (kp - 64);
            }
        }
        uint64_t x0 = 0, x1 = 0;  // u[info_set] = msg, x = u G (polar.py:17-29,106-119)
        for (int k = 0; k < nb; ++k) {
            const uint32_t v = (uint32_t)(((k < 8 ? m0 : m1) >> (8 * (k & 7))) & 255u);
            x0 ^= P.xtab[(k * 256 + v) * 2];
            x1 ^= P.xtab[(k * 256 + v) * 2 + 1];
        }
        if (P.msg && idx < P.B) {
            P.msg[idx * P.W] = m0;
            if (P.W > 1) P.msg[idx * P.W + 1] = m1;
        }
        if (P.unc_counters) {  // uncoded BPSK of the payload (kp <= 128 here: one payload block)
            int berr = 0;
            if (idx < P.B) {
                const uint64_t p0 = ((uint64_t)rb.y << 32) | rb.x, p1 = ((uint64_t)rb.w << 32) | rb.z;
                for (int c = 0; 2 * c < kp; ++c) {
                    const u32x4 rn = philox4x32(u32x4{(uint32_t)fr, (uint32_t)(fr >> 32), 0x40000000u + (uint32_t)c, 0u}, k0, k1);
                    double z[2];
                    bm_pair(((uint64_t)rn.y << 32) | rn.x, ((uint64_t)rn.w << 32) | rn.z, z[0], z[1]);
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int q = 2 * c + h;
                        if (q < kp) {
                            const int bit = (int)(((q < 64 ? p0 : p1) >> (q & 63)) & 1ULL);
                            const double y = (bit ? -1.0 : 1.0) + P.unc_sigma * z[h];
                            berr += (y < 0.0 ? 1 : 0) != bit;
                        }
                    }
                }
            }
            ufe += berr ? 1 : 0;
            ube += berr;
        }
        // ---- B: AWGN per frame, 2 symbols per lane per Philox block (NR: symbol p = x[order[p % N]])
        const int nf = (P.B - base) < 64 ? (int)(P.B - base) : 64;
        for (int j = 0; j < nf; ++j) {
            const uint64_t fj = (uint64_t)(P.frame0 + base + j);
            const uint64_t xa = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(x0 >> 32), j) << 32) |
                                (uint32_t)__builtin_amdgcn_readlane((uint32_t)x0, j);
            const uint64_t xb = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(x1 >> 32), j) << 32) |
                                (uint32_t)__builtin_amdgcn_readlane((uint32_t)x1, j);
            double* row = P.llr + (base + j) * E;
            for (int q = 0; q * 128 < E; ++q) {
                const u32x4 rn = philox4x32(u32x4{(uint32_t)fj, (uint32_t)(fj >> 32), (uint32_t)(lane + 64 * q), 0u}, k0, k1);
                double z[2];
                bm_pair(((uint64_t)rn.y << 32) | rn.x, ((uint64_t)rn.w << 32) | rn.z, z[0], z[1]);
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int p = lane + 64 * h + 128 * q;
                    if (p < E) {
                        const int pos = P.rm_E ? P.rm_order[p % P.N] : p;
                        const uint64_t xw = pos < 64 ? xa : xb;
                        const double sym = ((xw >> (pos & 63)) & 1) ? -1.0 : 1.0;
                        row[p] = (sym + P.sigma * z[h]) * P.llr_scale;
                    }
                }
            }
        }
    }
    if (P.unc_counters) {
        // one atomic per counter and workgroup: per-wave atomics on two words serialised at the L2
        // (15.6 k wavefronts per 10^6 frames; the fused launch took 0.55 ms against 0.27 without)
        __shared__ int part[4][2];
        const int fe = pscl::wave_sum(ufe), be = pscl::wave_sum(ube);
        if (lane == 0) {
            part[wave][0] = fe;
            part[wave][1] = be;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            const int tf = part[0][0] + part[1][0] + part[2][0] + part[3][0];
            const int tb = part[0][1] + part[1][1] + part[2][1] + part[3][1];
            unsigned long long* C = reinterpret_cast<unsigned long long*>(P.unc_counters);
            if (tf) atomicAdd(C + PSCL_CNT_FRAME_ERR, (unsigned long long)tf);
            if (tb) atomicAdd(C + PSCL_CNT_BIT_ERR, (unsigned long long)tb);
        }
    }
}

}  // namespace

// Rows of the fused TX (scl128_lane.hip TXF, pscl_simulate_device): the lane kernel draws the rows it
// decodes without writing them; the frames other decodes read again -- the deferred ones (exact
// re-decode) and the failing ones (DL-SCL retry chain) -- get channel_kernel's row written here,
// one wavefront per listed frame (lane c = Box-Muller pair c: positions c and c + 64), the codeword
// formed by every lane (channel_kernel phase A).  list[i] < count frames, at frame counter
// frame0 + list[i], row rows + list[i] * 128.
__global__ void __launch_bounds__(256) tx_rows_kernel(const pscl_decode_params P, const int64_t* __restrict__ list,
                                                      const int32_t* __restrict__ count, int64_t cap, double* rows,
                                                      int64_t frame0) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int64_t n = *count;
    if (n > cap) n = cap;
    for (int64_t i = (int64_t)blockIdx.x * 4 + wave; i < n; i += (int64_t)gridDim.x * 4) {  // wave-uniform
        const int64_t b = list[i];
        const uint64_t fr = (uint64_t)(frame0 + b);
        const u32x4 rb = philox4x32(u32x4{(uint32_t)fr, (uint32_t)(fr >> 32), 0xffffffffu, 0u}, P.tx_k0, P.tx_k1);
        const uint64_t r0 = ((uint64_t)rb.y << 32) | rb.x, r1 = ((uint64_t)rb.w << 32) | rb.z;
        const int kp = P.tx_kp, nbp = (kp + 7) >> 3, nb = (P.K + 7) >> 3;
        uint64_t m0 = kp >= 64 ? r0 : (r0 & ((1ULL << kp) - 1));
        uint64_t m1 = kp > 64 ? (r1 & ((kp >= 128) ? ~0ULL : ((1ULL << (kp - 64)) - 1))) : 0;
        uint32_t rem = 0;
        for (int k = 0; k < nbp; ++k) rem ^= P.tx_crctab[k * 256 + (uint32_t)(((k < 8 ? m0 : m1) >> (8 * (k & 7))) & 255u)];
        if (P.tx_crc_deg) {
            const uint64_t rw = (uint64_t)rem;
            if (kp < 64) {
                m0 |= rw << kp;
                if (kp + P.tx_crc_deg > 64) m1 |= rw >> (64 - kp);
            } else {
                m1 |= rw << (kp - 64);
            }
        }
        uint64_t x0 = 0, x1 = 0;
        for (int k = 0; k < nb; ++k) {
            const uint32_t v = (uint32_t)(((k < 8 ? m0 : m1) >> (8 * (k & 7))) & 255u);
            x0 ^= P.tx_xtab[(k * 256 + v) * 2];
            x1 ^= P.tx_xtab[(k * 256 + v) * 2 + 1];
        }
        const u32x4 rn = philox4x32(u32x4{(uint32_t)fr, (uint32_t)(fr >> 32), (uint32_t)lane, 0u}, P.tx_k0, P.tx_k1);
        double z[2];
        bm_pair(((uint64_t)rn.y << 32) | rn.x, ((uint64_t)rn.w << 32) | rn.z, z[0], z[1]);
        double* row = rows + b * 128;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const double sym = (((h ? x1 : x0) >> lane) & 1ULL) ? -1.0 : 1.0;
            row[lane + 64 * h] = (sym + P.tx_sigma * z[h]) * P.tx_scale;
        }
    }
}

// ------------------------------------------------------------------------- launchers

hipError_t pscl_launch_tx_rows(const pscl_decode_params& P, const int64_t* list, const int32_t* count, int64_t cap,
                               double* rows, int64_t frame0, hipStream_t s) {
    if (cap <= 0) return hipSuccess;
    int64_t grid = (cap + 3) / 4;
    if (grid > 1024) grid = 1024;  // (the count is read on the device; few frames in practice)
    hipLaunchKernelGGL(tx_rows_kernel, dim3((unsigned)grid), dim3(256), 0, s, P, list, count, cap, rows, frame0);
    return hipGetLastError();
}

// wavefronts per workgroup: the choice that keeps the most wavefronts resident per CU
// under the 160 KB LDS budget (each workgroup also holds the 2 KB exp table); 0 if none fits
int pscl_decode_wpg(const pscl_decode_params& P) {
    if (P.long_mode) return 1;  // one wavefront per workgroup, state in global scratch
    const int cu_lds = 160 * 1024, tbl = P.wg_fixed_bytes;
    int best = 0, best_res = 0;
    // workgroup size cap (tuning knob PSCL_TUNE_RETRY_WPG, set on the DL-SCL retry launches)
    const int wmax = P.wpg_cap >= 1 && P.wpg_cap < PSCL_MAX_WAVES_PER_WG ? P.wpg_cap : PSCL_MAX_WAVES_PER_WG;
    for (int w = 1; w <= wmax; ++w) {
        const int wg = tbl + w * P.wave_bytes;
        if (wg > cu_lds) break;
        int res = (cu_lds / wg) * w;
        if (res > 32) res = 32;
        if (res >= best_res) {
            best_res = res;
            best = w;
        }
    }
    return best;
}

static int decode_lds_bytes(const pscl_decode_params& P, int hist) {
    (void)hist;
    return P.wg_fixed_bytes + pscl_decode_wpg(P) * P.wave_bytes;
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
    if (P.long_mode) return pscl_long_grid(P.grid_cap > 0 && P.grid_cap < P.B ? P.grid_cap : P.B, P.L);
    const int per_wg = pscl_decode_wpg(P) * (32 / pscl_decode_lmax(P.L));  // frames per workgroup
    int64_t g = (P.B + per_wg - 1) / per_wg;
    // (counting launches, P.ref: at most PSCL_COUNT_GRID workgroups, whose wavefronts stride over
    // frames and add their counts once at the end)
    const int64_t cmax = P.ref && !P.cpart ? PSCL_COUNT_GRID : (1 << 20);
    const int64_t cap = P.grid_cap > 0 && P.grid_cap < cmax ? P.grid_cap : cmax;
    return g < 1 ? 1 : (g > cap ? cap : g);
}

void pscl_decode_layout(pscl_decode_params& P, int hist) {
    const int lmax = pscl_decode_lmax(P.L);
    P.long_mode = P.N > PSCL_FAST_N ? 1 : 0;
    if (P.long_mode) {
        P.fast = 0;
        P.wg_fixed_bytes = P.wave_bytes = P.a_bytes = 0;
        P.long_block_bytes = pscl_long_block_bytes(P.N, P.L, P.K, hist);
        return;
    }
    const int F = 32 / lmax;  // frames per wavefront
    P.fast = (P.N == 128 && P.L <= 8) ? 1 : 0;
    // exp table (exact metric tails; the screening launch, P.apx, has none) + scl128 epilogue tables
    P.wg_fixed_bytes = (P.apx ? 0 : PSCL_EXP_TABLE_WORDS * 8) + (P.fast && PSCL_EPI_LDS ? P.epi_words * 8 : 0);
    if (P.fast) P.wg_fixed_bytes = (P.wg_fixed_bytes + 255) & ~255;  // frames start on LDS bank 0 (Layout128)
    if (P.fast) {
        P.a_bytes = F * pscl_fast128_fstride(P.L, P.rm_E != 0) * 8;
        const int wb = P.a_bytes + (hist ? F * P.K * P.L * 9 : 0);
        P.wave_bytes = (wb + 15) & ~15;
    } else {
        const int fstride = P.N + (P.N >= 8 ? P.L * (P.N / 2 - 2) : 0);  // doubles per frame
        P.a_bytes = F * fstride * 8;
        const int wb = P.a_bytes + 64 + (hist ? F * (P.K * P.L * 8 + P.N * P.L) : 0);
        P.wave_bytes = (wb + 15) & ~15;
    }
}

// the screening launch of an N = 128 code without a compiled-in screening kernel (any information
// set, L = 4, 8 or 16): the runtime-information-set lane-per-path kernel (scl_lane_long.hip at n = 7)
static bool lane_long128(const pscl_decode_params& P) {
    return P.N == 128 && !P.long_mode && P.apx && !pscl_screening_available(P) && pscl_lane_long_available(P);
}

int pscl_lane_long128_available(const pscl_decode_params& P) { return lane_long128(P) ? 1 : 0; }

hipError_t pscl_launch_decode(const pscl_decode_params& P, int hist, hipStream_t s) {
    if (P.long_mode) {
        if (!hist && P.apx) return pscl_launch_lane_long(P, s);  // (screening: lane-per-path only)
        return pscl_launch_long(P, hist, s);
    }
    if (!hist && pscl_lane_available(P)) {  // one wavefront of 64 / L frames per workgroup
        const int fw = pscl_lane_frames_per_wg(P.L);
        const int64_t g = (P.B + fw - 1) / fw;
        // (counting launches with atomics: at most PSCL_LANE_COUNT_GRID wavefronts, each adding its
        // frames' counts with one atomic per counter when it ends)
        const int64_t cap = P.ref && !P.cpart ? PSCL_LANE_COUNT_GRID : (1 << 20);
        return pscl_launch_lane(P, g < 1 ? 1 : (g > cap ? cap : g), s);
    }
    if (!hist && pscl_lane_fs_available(P)) {  // (P.B: the round's entry capacity)
        const int fw = pscl_lane_frames_per_wg(P.L);
        const int64_t g = (P.B + fw - 1) / fw;
        return pscl_launch_lane_fs(P, g < 1 ? 1 : (g > (1 << 20) ? (1 << 20) : g), s);
    }
    if (!hist && lane_long128(P)) return pscl_launch_lane_long(P, s);
    if (!hist && pscl_lane_exact_available(P)) return pscl_launch_lane_exact(P, s);
    if (pscl_decode_wpg(P) < 1) return hipErrorInvalidValue;
    const int64_t grid = pscl_decode_grid(P);
    if (P.fast) return pscl_launch_decode128(P, hist, pscl_decode_wpg(P), grid, decode_lds_bytes(P, hist), s);
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

int64_t pscl_decode_count_slots(const pscl_decode_params& P0, int hist) {
    if (!P0.ref || P0.out_by_row || hist) return 0;
    pscl_decode_params P = P0;
    P.cpart = reinterpret_cast<int32_t*>(16);  // (the grids of a launch that stores its counts)
    if (P.long_mode) return P.apx && pscl_lane_long_available(P) ? pscl_lane_long_grid(P) : 0;
    if (pscl_lane_available(P)) {
        const int fw = pscl_lane_frames_per_wg(P.L);
        const int64_t g = (P.B + fw - 1) / fw;
        return g < 1 ? 1 : (g > (1 << 20) ? (1 << 20) : g);
    }
    if (lane_long128(P)) return pscl_lane_long_grid(P);
    if (pscl_lane_exact_available(P)) return pscl_lane_exact_grid(P);
    if (!P.fast || pscl_decode_wpg(P) < 1) return 0;  // (the generic kernel adds per frame)
    return pscl_decode_grid(P) * pscl_decode_wpg(P);
}

namespace {
__global__ void __launch_bounds__(256) count_reduce_kernel(int4* __restrict__ part, int64_t n, int64_t* counters) {
    __shared__ long long acc[4][4];
    long long a = 0, b = 0, c = 0, d = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const int4 v = part[i];
        a += v.x;
        b += v.y;
        c += v.z;
        d += v.w;
        if (v.x | v.y | v.z | v.w) part[i] = make_int4(0, 0, 0, 0);  // (zero for the next launch)
    }
#pragma unroll
    for (int sft = 32; sft >= 1; sft >>= 1) {
        a += __shfl_xor(a, sft);
        b += __shfl_xor(b, sft);
        c += __shfl_xor(c, sft);
        d += __shfl_xor(d, sft);
    }
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        acc[wave][0] = a;
        acc[wave][1] = b;
        acc[wave][2] = c;
        acc[wave][3] = d;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        const long long t = acc[0][threadIdx.x] + acc[1][threadIdx.x] + acc[2][threadIdx.x] + acc[3][threadIdx.x];
        static constexpr int idx[4] = {PSCL_CNT_FRAME_ERR, PSCL_CNT_BIT_ERR, PSCL_CNT_PAYLOAD_ERR, PSCL_CNT_PAYLOAD_BIT};
        if (t) atomicAdd(reinterpret_cast<unsigned long long*>(counters) + idx[threadIdx.x], (unsigned long long)t);
    }
}
}  // namespace

hipError_t pscl_launch_count_reduce(int32_t* cpart, int64_t slots, int64_t* counters, hipStream_t s) {
    if (slots <= 0) return hipSuccess;
    int64_t g = (slots + 2047) / 2048;  // ~8 slots per thread
    if (g > 256) g = 256;
    hipLaunchKernelGGL(count_reduce_kernel, dim3((unsigned)g), dim3(256), 0, s, reinterpret_cast<int4*>(cpart), slots,
                       counters);
    return hipGetLastError();
}

// uncoded BPSK baseline: one frame per lane, kp payload symbols, errors reduced per block
// TX chain of the long codes (N > PSCL_FAST_N): one wavefront per frame, lane w holds word w
// of the message (w < W) and of the codeword (w < N / 64).  Same stream as channel_kernel:
// payload bits 128 j .. 128 j + 127 from the Philox block (frame, 0xffffffff - j) (j = 0 is
// channel_kernel's block), symbol noise from the blocks (frame, lane + 64 q).
__global__ void __launch_bounds__(256) channel_long_kernel(const pscl_channel_params P) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t k0 = (uint32_t)P.seed, k1 = (uint32_t)(P.seed >> 32) ^ (P.stream_id * 0x85EBCA6Bu);
    const int E = P.rm_E ? P.rm_E : P.N;
    const int kp = P.k_payload, W = P.W, NW = P.N >> 6;
    const int nb = (P.K + 7) >> 3, nbp = (kp + 7) >> 3;
    for (int64_t idx = (int64_t)blockIdx.x * 4 + wave; idx < P.B; idx += (int64_t)gridDim.x * 4) {  // wave-uniform
        const uint64_t fr = (uint64_t)(P.frame0 + idx);
        // payload word `lane`, masked to kp bits
        uint64_t m = 0;
        if (lane < W) {
            const u32x4 rb = philox4x32(u32x4{(uint32_t)fr, (uint32_t)(fr >> 32), 0xffffffffu - (uint32_t)(lane >> 1), 0u},
                                        k0, k1);
            m = (lane & 1) ? (((uint64_t)rb.w << 32) | rb.z) : (((uint64_t)rb.y << 32) | rb.x);
            const int nbits = kp - 64 * lane;
            m = nbits >= 64 ? m : (nbits > 0 ? (m & ((1ULL << nbits) - 1)) : 0ULL);
        }
        // attach_cols (crc.py:19-37): the remainder of the payload bytes, XOR-reduced over lanes
        uint32_t rem = 0;
        if (lane < W)
            for (int t = 0; t < 8; ++t) {
                const int k = 8 * lane + t;
                if (k < nbp) rem ^= P.crctab[k * 256 + (uint32_t)((m >> (8 * t)) & 255u)];
            }
        for (int sft = 1; sft < 64; sft <<= 1) rem ^= (uint32_t)__shfl_xor((int)rem, sft);
        if (P.crc_deg) {
            const int w0 = kp >> 6, o = kp & 63;
            if (lane == w0) m |= (uint64_t)rem << o;
            if (lane == w0 + 1 && o + P.crc_deg > 64) m |= (uint64_t)rem >> (64 - o);
        }
        // codeword x = u G (polar.py:17-29,106-119): one table row per message byte
        uint64_t x = 0;
        for (int k = 0; k < nb; ++k) {
            const uint64_t mw = pscl::shfl_u64(m, k >> 3);
            const uint32_t v = (uint32_t)((mw >> (8 * (k & 7))) & 255u);
            if (lane < NW) x ^= P.xtab[((size_t)k * 256 + v) * NW + lane];
        }
        if (P.msg && lane < W) P.msg[idx * W + lane] = m;
        double* row = P.llr + idx * E;
        for (int q = 0; q * 128 < E; ++q) {
            const u32x4 rn = philox4x32(u32x4{(uint32_t)fr, (uint32_t)(fr >> 32), (uint32_t)(lane + 64 * q), 0u}, k0, k1);
            double z[2];
            bm_pair(((uint64_t)rn.y << 32) | rn.x, ((uint64_t)rn.w << 32) | rn.z, z[0], z[1]);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int p = lane + 64 * h + 128 * q;
                const int pos = p < E ? (P.rm_E ? P.rm_order[p % P.N] : p) : 0;
                const uint64_t xw = pscl::shfl_u64(x, pos >> 6);  // (every lane takes part)
                if (p < E) {
                    const double sym = ((xw >> (pos & 63)) & 1) ? -1.0 : 1.0;
                    row[p] = (sym + P.sigma * z[h]) * P.llr_scale;
                }
            }
        }
    }
}

__global__ void __launch_bounds__(256) uncoded_kernel(const pscl_channel_params P, int64_t* counters) {
    __shared__ long long part[4][2];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t k0 = (uint32_t)P.seed, k1 = (uint32_t)(P.seed >> 32) ^ (P.stream_id * 0x85EBCA6Bu);
    const int kp = P.k_payload;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int ferr = 0, berr = 0;
    if (idx < P.B) {
        const uint64_t fr = (uint64_t)(P.frame0 + idx);
        u32x4 rb = philox4x32(u32x4{(uint32_t)fr, (uint32_t)(fr >> 32), 0xffffffffu, 0u}, k0, k1);
        uint64_t r0 = ((uint64_t)rb.y << 32) | rb.x, r1 = ((uint64_t)rb.w << 32) | rb.z;
        for (int c = 0; 2 * c < kp; ++c) {
            if (c && (c & 63) == 0) {  // payload bits 128 j.. (long codes): Philox block (frame, 0xffffffff - j)
                rb = philox4x32(u32x4{(uint32_t)fr, (uint32_t)(fr >> 32), 0xffffffffu - (uint32_t)(c >> 6), 0u}, k0, k1);
                r0 = ((uint64_t)rb.y << 32) | rb.x;
                r1 = ((uint64_t)rb.w << 32) | rb.z;
            }
            const u32x4 rn = philox4x32(u32x4{(uint32_t)fr, (uint32_t)(fr >> 32), 0x40000000u + (uint32_t)c, 0u}, k0, k1);
            double z[2];
            bm_pair(((uint64_t)rn.y << 32) | rn.x, ((uint64_t)rn.w << 32) | rn.z, z[0], z[1]);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int q = 2 * c + h;
                if (q < kp) {
                    const int bit = (int)((((q & 127) < 64 ? r0 : r1) >> (q & 63)) & 1ULL);
                    const double y = (bit ? -1.0 : 1.0) + P.sigma * z[h];
                    berr += (y < 0.0 ? 1 : 0) != bit;  // (2 y / var < 0 <=> y < 0: var > 0)
                }
            }
        }
        ferr = berr ? 1 : 0;
    }
    ferr = pscl::wave_sum(ferr);
    berr = pscl::wave_sum(berr);
    if (lane == 0) {
        part[wave][0] = ferr;
        part[wave][1] = berr;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        long long t = 0;
        for (int w = 0; w < 4; ++w) t += part[w][threadIdx.x];
        unsigned long long* C = reinterpret_cast<unsigned long long*>(counters);
        if (t) atomicAdd(C + (threadIdx.x == 0 ? PSCL_CNT_FRAME_ERR : PSCL_CNT_BIT_ERR), (unsigned long long)t);
        if (threadIdx.x == 0 && blockIdx.x == 0) atomicAdd(C + PSCL_CNT_FRAMES, (unsigned long long)P.B);
    }
}

hipError_t pscl_launch_uncoded(const pscl_channel_params& P, int64_t* counters, hipStream_t s) {
    hipLaunchKernelGGL(uncoded_kernel, dim3((unsigned)((P.B + 255) / 256)), dim3(256), 0, s, P, counters);
    return hipGetLastError();
}

// diagnostic: both metric-tail evaluations of the decode kernels on n values
__global__ void __launch_bounds__(256) softplus_tails_kernel(const double* v, int64_t n, const uint64_t* exp_table,
                                                              double* exact, double* apx) {
    __shared__ uint64_t T[PSCL_EXP_TABLE_WORDS];
    for (int i = threadIdx.x; i < PSCL_EXP_TABLE_WORDS; i += blockDim.x) T[i] = exp_table[i];
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double x = v[i];
        exact[i] = pscl_softplus_tail_bf(x, T);
        apx[i] = PSCL_TAIL_ABS ? pscl_softplus_tail_abs(x) : pscl_softplus_tail_scr(x);
    }
}

// diagnostic: max |pscl_tail_abs_f32(x32) - glibc tail(x32)| over the fp32 bit patterns
// [lo, hi] (the screening tail is a function of x32 = fl32(|v|) alone: glibc_softplus.h).
// out[0] = the largest error's fp64 bits (non-negative doubles order like their bit patterns),
// out[1] = (high word of that error << 32) | its x32 bit pattern, for the argmax.
// bits = 1: the bits form, max |pscl_tail2_f32(y32) - log1p(exp(-y32 ln 2)) / ln 2| (glibc_softplus.h)
__global__ void __launch_bounds__(256) tail_abs_scan_kernel(uint32_t lo, uint32_t hi, const uint64_t* exp_table,
                                                             unsigned long long* out, int bits) {
    __shared__ uint64_t T[PSCL_EXP_TABLE_WORDS];
    for (int i = threadIdx.x; i < PSCL_EXP_TABLE_WORDS; i += blockDim.x) T[i] = exp_table[i];
    __syncthreads();
    unsigned long long best = 0, key = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= hi; i += stride) {
        const float x32 = __uint_as_float((uint32_t)i);
        const double ex = bits ? pscl_softplus_tail_bf((double)x32 * PSCL_LOGE2, T) / PSCL_LOGE2
                               : pscl_softplus_tail_bf((double)x32, T);
        const double ap = bits ? (double)pscl_tail2_f32(x32) : (double)pscl_tail_abs_f32(x32);
        const unsigned long long eb = (unsigned long long)pscl_asu64(fabs(ap - ex));
        if (eb > best) {
            best = eb;
            key = ((eb >> 32) << 32) | (uint32_t)i;
        }
    }
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) {
        const unsigned long long ob = __shfl_xor(best, s), ok = __shfl_xor(key, s);
        best = ob > best ? ob : best;
        key = ok > key ? ok : key;
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMax(out, best);
        atomicMax(out + 1, key);
    }
}

hipError_t pscl_launch_tail_abs_scan(uint32_t lo, uint32_t hi, const uint64_t* exp_table, unsigned long long* out,
                                     hipStream_t s, int bits) {
    hipLaunchKernelGGL(tail_abs_scan_kernel, dim3(8192), dim3(256), 0, s, lo, hi, exp_table, out, bits);
    return hipGetLastError();
}

hipError_t pscl_launch_softplus_tails(const double* v, int64_t n, const uint64_t* exp_table, double* exact,
                                     double* apx, hipStream_t s) {
    int64_t grid = (n + 255) / 256;
    if (grid > 4096) grid = 4096;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(softplus_tails_kernel, dim3((unsigned)grid), dim3(256), 0, s, v, n, exp_table, exact, apx);
    return hipGetLastError();
}

hipError_t pscl_launch_channel(const pscl_channel_params& P, hipStream_t s) {
    int64_t grid = (P.B + 255) / 256;
    // (with the uncoded baseline fused: 2048 workgroups, each counting over several strides)
    const int64_t gcap = P.unc_counters ? 2048 : (1 << 20);
    if (grid > gcap) grid = gcap;
    if (grid < 1) grid = 1;
    if (P.N > PSCL_FAST_N) {  // one wavefront per frame
        int64_t g = (P.B + 3) / 4;
        if (g > (1 << 16)) g = 1 << 16;
        hipLaunchKernelGGL(channel_long_kernel, dim3((unsigned)g), dim3(256), 0, s, P);
    } else {
        hipLaunchKernelGGL(channel_kernel, dim3((unsigned)grid), dim3(256), 0, s, P);
    }
    return hipGetLastError();
}
