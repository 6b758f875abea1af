// scl_cpu.cpp -- the product's host (CPU) SC/SCL decoder: decode_scl
// (dl_scl_polar/polar/scl.py:108-209) for hosts without a GPU (BASELINE config 1: SC, M = 1,
// 1000 frames through run_fer_sweep "on CPU", run_fer_sweep.py:41-191).  Same contract and
// outputs as pscl_decode (include/polar_scl.h), bit for bit: the f/g tree in fp64 (polar.py:
// 122-127), the path metric with the glibc port of exp/log1p (glibc_softplus.h, as the GPU
// kernels), Python's stable list sort (scl.py:173-174), first CRC-passing candidate (scl.py:
// 190-198).  No GPU and no HIP call: the frames of a batch are split over host threads.
//
// Layout (per thread, reused across frames): depth d = 1..n of the LLR tree holds L slots of
// N >> d values; a path at list position p writes every depth its phase rewrites into slot p and
// reads the first rewritten depth's parent through its slot table -- all paths rewrite the same
// depths at a phase (SC is lockstep), so no slot another path still needs is overwritten, and a
// clone copies its parent's table (n bytes), never LLR values.  Decided bits: one byte per phase.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <thread>
#include <vector>

#include "glibc_softplus.h"
#include "polar_scl.h"

namespace {

const uint64_t kExpTableCpu[256] = {
#include "exp_table.inc"
};

// np.sign(a) * np.sign(b) * np.minimum(|a|, |b|) (polar.py:122-123), signed zeros included:
// np.sign(+-0) = +0, so a zero result takes the sign of the nonzero operand (+0 if both are zero)
double f_node(double a, double b) {
    const double m = fabs(a) < fabs(b) ? fabs(a) : fabs(b);
    if (a == 0.0 || b == 0.0) return (a == 0.0 && b == 0.0) ? 0.0 : std::copysign(0.0, a == 0.0 ? b : a);
    return (std::signbit(a) != std::signbit(b)) ? -m : m;
}
double g_node(double a, double b, int c) { return b + (c ? -a : a); }  // b + (1 - 2c) a, polar.py:126-127

// metric + np.logaddexp(0, +-llr) (scl.py:102-105): npy_logaddexp(0, v) with glibc exp/log1p
double metric_add(double metric, double llr, int bit) {
    const double v = bit ? llr : -llr;
    const double t = pscl_softplus_tail(v, kExpTableCpu);
    return metric + pscl_logaddexp0(v, t);
}

struct Cand {
    double metric;
    int parent, bit;
};

struct CpuScl {
    int N, n, K, L, deg;
    uint64_t poly;
    std::vector<uint8_t> is_info;
    std::vector<int32_t> info;
    std::vector<double> alpha;  // [n + 1][L][N] (depth d uses N >> d of each slot's N)
    // per list position, two generations (current / next list)
    std::vector<uint8_t> u[2], tab[2];
    std::vector<double> il[2], met[2];
    std::vector<Cand> cand;
    std::vector<uint8_t> x;

    CpuScl(int N_, const int32_t* info_set, int K_, int L_, uint64_t poly_)
        : N(N_), n(__builtin_ctz((unsigned)N_)), K(K_), L(L_), deg(0), poly(poly_) {
        if (poly) deg = 63 - __builtin_clzll(poly);
        is_info.assign(N, 0);
        info.assign(info_set, info_set + K);
        for (int i = 0; i < K; ++i) is_info[info_set[i]] = 1;
        alpha.assign((size_t)(n + 1) * L * N, 0.0);
        for (int s = 0; s < 2; ++s) {
            u[s].assign((size_t)L * N, 0);
            tab[s].assign((size_t)L * (n + 1), 0);
            il[s].assign((size_t)L * (K ? K : 1), 0.0);
            met[s].assign(L, 0.0);
        }
        cand.reserve(2 * L);
        x.assign(N, 0);
    }

    double* slot(int d, int s) { return alpha.data() + ((size_t)d * L + s) * N; }

    // partial sums of the w-bit left sibling u[lo, lo + w): x = u G_w (natural order)
    void transform(const uint8_t* useg, int w) {
        memcpy(x.data(), useg, (size_t)w);
        for (int h = 1; h < w; h <<= 1)
            for (int i = 0; i < w; i += 2 * h)
                for (int j = i; j < i + h; ++j) x[j] ^= x[j + h];
    }

    bool crc_ok(const uint8_t* bits) const {  // crc.py:40-56: remainder of the K-bit message
        if (!poly) return true;
        uint64_t rem = 0;
        for (int i = 0; i < K; ++i) {
            rem = (rem << 1) | bits[i];
            if ((rem >> deg) & 1) rem ^= poly;
        }
        return rem == 0;
    }

    // one frame; outputs as pscl_decode (row pointers, any may be null)
    void decode(const double* llr, const int8_t* force, int32_t* n_paths, int8_t* best_bits, uint8_t* crc_pass,
                int32_t* best_idx, double* metrics, int8_t* cands, double* info_llrs) {
        memcpy(slot(0, 0), llr, sizeof(double) * (size_t)N);
        int cur = 0, cnt = 1, j = 0;
        met[0][0] = 0.0;
        for (int phi = 0; phi < N; ++phi) {
            const int start = phi ? n - __builtin_ctz((unsigned)phi) : 1;
            cand.clear();
            const bool info_phase = is_info[phi] != 0;
            const int fbit = (info_phase && force) ? force[j] : -1;
            for (int p = 0; p < cnt; ++p) {
                uint8_t* tp = tab[cur].data() + (size_t)p * (n + 1);
                const uint8_t* up = u[cur].data() + (size_t)p * N;
                for (int d = start; d <= n; ++d) {
                    const int w = N >> d, k = phi >> (n - d);
                    const double* P = d == 1 ? slot(0, 0) : slot(d - 1, tp[d - 1]);
                    tp[d] = (uint8_t)p;
                    double* o = slot(d, p);
                    if (!(k & 1)) {
                        for (int i = 0; i < w; ++i) o[i] = f_node(P[i], P[i + w]);
                    } else {
                        transform(up + (size_t)(k - 1) * w, w);
                        for (int i = 0; i < w; ++i) o[i] = g_node(P[i], P[i + w], x[i]);
                    }
                }
                const double lam = slot(n, p)[0];
                if (info_phase) il[cur][(size_t)p * (K ? K : 1) + j] = lam;  // decision LLR (scl.py:158,166)
                const double m = met[cur][p];
                if (!info_phase) {
                    cand.push_back({metric_add(m, lam, 0), p, 0});
                } else if (fbit == 0 || fbit == 1) {
                    cand.push_back({metric_add(m, lam, fbit), p, fbit});
                } else {
                    cand.push_back({metric_add(m, lam, 0), p, 0});
                    cand.push_back({metric_add(m, lam, 1), p, 1});
                }
            }
            // python's list.sort(key=metric): stable (scl.py:173); keep the first L (scl.py:174)
            std::stable_sort(cand.begin(), cand.end(), [](const Cand& a, const Cand& b) { return a.metric < b.metric; });
            const int ncnt = (int)std::min<size_t>(cand.size(), (size_t)L);
            const int nxt = cur ^ 1;
            const size_t KW = K ? K : 1;
            for (int q = 0; q < ncnt; ++q) {
                const Cand& c = cand[q];
                memcpy(tab[nxt].data() + (size_t)q * (n + 1), tab[cur].data() + (size_t)c.parent * (n + 1), (size_t)n + 1);
                memcpy(u[nxt].data() + (size_t)q * N, u[cur].data() + (size_t)c.parent * N, (size_t)phi);
                u[nxt][(size_t)q * N + phi] = (uint8_t)c.bit;
                if (info_phase) memcpy(il[nxt].data() + q * KW, il[cur].data() + (size_t)c.parent * KW, sizeof(double) * (size_t)(j + 1));
                else if (j) memcpy(il[nxt].data() + q * KW, il[cur].data() + (size_t)c.parent * KW, sizeof(double) * (size_t)j);
                met[nxt][q] = c.metric;
            }
            // the slots written this phase belong to list positions of the OLD list: survivors moved
            // to new positions keep pointing at their parent's slots through the copied tables
            // (depths >= start are rewritten by every path at the next phase that needs them)
            cur = nxt;
            cnt = ncnt;
            if (info_phase) ++j;
        }
        // epilogue (scl.py:176-209): candidates u[info_set] in list order, first CRC pass
        std::vector<uint8_t> bits((size_t)K);
        int best = -1;
        for (int p = 0; p < cnt; ++p) {
            const uint8_t* up = u[cur].data() + (size_t)p * N;
            for (int i = 0; i < K; ++i) bits[i] = up[info[i]];
            if (cands)
                for (int i = 0; i < K; ++i) cands[(size_t)p * K + i] = (int8_t)bits[i];
            if (metrics) metrics[p] = met[cur][p];
            if (info_llrs) memcpy(info_llrs + (size_t)p * K, il[cur].data() + (size_t)p * (K ? K : 1), sizeof(double) * (size_t)K);
            if (best < 0 && poly && crc_ok(bits.data())) best = p;
        }
        const bool pass = best >= 0 || !poly;
        if (best < 0) best = 0;
        const uint8_t* ub = u[cur].data() + (size_t)best * N;
        if (best_bits)
            for (int i = 0; i < K; ++i) best_bits[i] = (int8_t)ub[info[i]];
        if (crc_pass) *crc_pass = pass ? 1 : 0;
        if (best_idx) *best_idx = best;
        if (n_paths) *n_paths = cnt;
    }
};

}  // namespace

extern "C" int pscl_decode_cpu(int N, const int32_t* info_set, int K, int L, uint64_t crc_poly, const double* llr,
                               int64_t B, const int8_t* forced, int32_t* n_paths, int8_t* best_bits, uint8_t* crc_pass,
                               int32_t* best_idx, double* metrics, int8_t* cands, double* info_llrs, int threads) {
    if (N < 2 || N > PSCL_MAX_N || (N & (N - 1))) return PSCL_EINVAL;
    if (L < 1 || L > 255 || K < 0 || K > N || B < 0 || (B && !llr) || (K && !info_set)) return PSCL_EINVAL;
    for (int i = 0; i < K; ++i)
        if (info_set[i] < 0 || info_set[i] >= N || (i && info_set[i] <= info_set[i - 1])) return PSCL_EINVAL;
    if (crc_poly) {
        const int deg = 63 - __builtin_clzll(crc_poly);
        if (deg <= 0 || K <= deg) return PSCL_EINVAL;  // crc.py:50-51 (message too short)
    }
    if (forced)
        for (int64_t i = 0; i < B * K; ++i)
            if (forced[i] < -1 || forced[i] > 1) return PSCL_EINVAL;
    if (B == 0) return PSCL_OK;
    int T = threads > 0 ? threads : (int)std::thread::hardware_concurrency();
    if (T < 1) T = 1;
    if ((int64_t)T > B) T = (int)B;
    auto work = [&](int t) {
        CpuScl dec(N, info_set, K, L, crc_poly);
        const int64_t b0 = B * t / T, b1 = B * (t + 1) / T;
        for (int64_t b = b0; b < b1; ++b)
            dec.decode(llr + b * N, forced ? forced + b * K : nullptr, n_paths ? n_paths + b : nullptr,
                       best_bits ? best_bits + b * K : nullptr, crc_pass ? crc_pass + b : nullptr,
                       best_idx ? best_idx + b : nullptr, metrics ? metrics + b * L : nullptr,
                       cands ? cands + b * L * K : nullptr, info_llrs ? info_llrs + b * L * K : nullptr);
    };
    if (T == 1) {
        work(0);
    } else {
        std::vector<std::thread> pool;
        for (int t = 0; t < T; ++t) pool.emplace_back(work, t);
        for (auto& th : pool) th.join();
    }
    return PSCL_OK;
}
