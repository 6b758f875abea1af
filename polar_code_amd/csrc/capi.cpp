// capi.cpp -- C ABI of libpolar_mi355x.so (declared in include/polar_scl.h).
//
// Host side of the engine: validates arguments with the reference's error semantics
// (scl.py:117-131, crc.py:40-49), precomputes the per-code constants (information mask,
// CRC syndrome/remainder columns, glibc exp table), owns device scratch and the stream,
// and launches the kernels in scl_kernels.hip.  Every handle entry point runs on the GPU and
// fails with PSCL_EDEVICE when no GPU is present; the product's host decoder for GPU-less runs
// is the handle-free pscl_decode_cpu (scl_cpu.cpp).
#include <hip/hip_runtime.h>
#include <math.h>

#include <cmath>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <string>
#include <utility>
#include <vector>

#include "polar_scl.h"
#include "scl_kernels.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                     \
    do {                                                                                  \
        hipError_t _e = (expr);                                                           \
        if (_e != hipSuccess)                                                             \
            return fail(_e == hipErrorOutOfMemory ? PSCL_ENOMEM : PSCL_EDEVICE, "%s: %s", \
                        #expr, hipGetErrorString(_e));                                    \
    } while (0)

#ifndef PSCL_BUILD_HASH
#define PSCL_BUILD_HASH "unhashed"
#endif
// marker + hash, found in the .so bytes by polar_code_amd/build.py's staleness check
__attribute__((used)) const char kBuildHash[] = "PSCL_BUILD_HASH=" PSCL_BUILD_HASH;

const uint64_t kExpTable[256] = {
#include "exp_table.inc"
};

// MSB-first bits of the polynomial value (crc.py:10-16); returns degree
int poly_degree(uint64_t poly) {
    int len = 0;
    for (uint64_t v = poly; v; v >>= 1) len++;
    return len - 1;
}

// remainder of bits[0..len) after the long division of crc.py (positions 0..len-deg-1
// are divided out); remainder bit i = buffer[len-deg+i]
uint32_t crc_remainder(const std::vector<uint8_t>& in, uint64_t poly, int deg) {
    std::vector<uint8_t> buf(in);
    const int len = (int)buf.size();
    for (int i = 0; i + deg < len; ++i) {
        if (!buf[i]) continue;
        for (int k = 0; k <= deg; ++k) buf[i + k] ^= (uint8_t)((poly >> (deg - k)) & 1);
    }
    uint32_t r = 0;
    for (int i = 0; i < deg; ++i)
        if (buf[len - deg + i]) r |= 1u << i;
    return r;
}

struct DevBuf {
    void* p = nullptr;
    size_t n = 0;
};

}  // namespace

// the arguments of a pscl_dlscl_device call (kept for a pipelined call's deferred chains)
struct pscl_dl_call {
    const double* d_llr = nullptr;
    int64_t B = 0;
    int rounds = 0;
    uint64_t* d_best = nullptr;
    uint8_t* d_flags = nullptr;
    int32_t* d_attempts = nullptr;
    int32_t* d_tried = nullptr;
    int tried_stride = 0;
    const uint64_t* d_ref = nullptr;
    int k_payload = 0;
    int64_t* d_counters_dl = nullptr;
    int64_t nch = 1, cap = 0;
    int nsplit = 2, pbase = 0;
    bool pipe = false;
};

// depth of the DL-SCL pipeline (pscl_set_pipelined): a pipelined call's compaction output and, for
// pscl_simulate_device, its TX buffers are one of kDlPar sets, rewritten only after the retry chains
// of the call kDlPar back have ended -- the handle's stream runs up to kDlPar - 1 calls ahead of
// the chains (2 measured 175 M frames/s on the config-3 sweep, the stream waiting on chains of the
// low-SNR points)
constexpr int kDlPar = 4;
// retry-chain sets: the chains of consecutive pipelined calls (and of consecutive chunks of one
// call) alternate two sets of streams, events and state, so a call's chains run beside the previous
// call's instead of queueing behind them; each set holds the chain pair of one call (k = 0, 1 at
// index 2 set + k)
constexpr int kChainSets = 2, kChainStreams = 2 * kChainSets;

struct pscl_handle {
    int device = 0;
    int N = 0, n = 0, K = 0, L = 0, W = 1, crc_deg = 0;
    uint64_t crc_poly = 0;
    uint64_t info_mask[2] = {0, 0};   // phases 0..127 (the N <= 128 kernels)
    std::vector<uint64_t> info_words;  // [N/64 or 1] every phase (scl_long.hip)
    uint64_t* d_info_words = nullptr;
    std::vector<int32_t> info_set;
    std::vector<uint32_t> check_cols;   // [K]
    std::vector<uint32_t> attach_cols;  // [K - deg]
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    uint32_t* d_check_cols = nullptr;
    uint32_t* d_attach_cols = nullptr;
    int32_t* d_info_set = nullptr;
    uint64_t* d_exp_table = nullptr;
    int rm_E = 0;                     // NR rate matching (0 = off)
    int32_t* d_rm_src = nullptr;      // [N] de-interleave gather index
    int32_t* d_rm_order = nullptr;    // [N] interleaver order
    DevBuf scratch[128];
    hipStream_t retry_stream[kChainStreams] = {};  // DL-SCL retry chains: [2 set + k], chain k of a call
    hipStream_t side_stream[kChainStreams] = {};   // their deferred-entry work (PSCL_TUNE_DL_SCREEN)
    // the side streams of the other pipelining mode (their priority differs, create_priority_stream),
    // kept across pscl_set_pipelined switches: a stream creation costs ~0.5 ms of host time
    hipStream_t stash_pipe = nullptr, stash_retry[kChainStreams] = {}, stash_side[kChainStreams] = {};
    hipEvent_t ev_scr[kChainStreams] = {}, ev_def[kChainStreams] = {};
    hipEvent_t ev_base[kDlPar] = {}, ev_retry[kDlPar] = {}, ev_join[kChainSets] = {};
    int32_t* h_count = nullptr;          // pinned: failing-frame counts of the chunk parities
    double* d_beta = nullptr;         // [K][K] DL-SCL flip metric (null = |L0|)
    float* d_beta32g[2] = {nullptr, nullptr};  // K = 64: fp32 beta, [K][G][K / G] for G = 8, 4 (fused post)
    std::vector<float> beta32g_host;
    double beta_absmax = 0.0;         // max |beta| (dl_post_kernel's certificate)
    std::vector<double> beta_host;    // staging of the last pscl_set_beta upload (stream-ordered copy)
    uint64_t* d_epi = nullptr;        // scl128 epilogue tables (gather + syndrome)
    uint64_t* d_xtab = nullptr;       // TX: codeword of each message byte value
    uint32_t* d_crctab = nullptr;     // TX: CRC remainder of each payload byte value
    int epi_words = 0;
    bool timing = false;
    bool screen = true;               // screening decode for plain decodes (pscl_set_screening)
    bool screened = false;            // a screening decode ran (scratch screened_slot holds its count)
    int screened_slot = 36;
    // pipelined plain decodes (pscl_set_pipelined): a screening decode's exact re-decode runs on
    // pipe_stream and overlaps the caller's next decode; the two alternate scratch parities
    // (deferred-frame count + list: slots 36/37 and 64/65), and every other entry point, and
    // pscl_join, order the pending re-decodes back into the handle's stream
    bool pipelined = false;
    hipStream_t pipe_stream = nullptr;
    hipEvent_t ev_pscr[2] = {nullptr, nullptr}, ev_px[2] = {nullptr, nullptr};
    bool px_pending[2] = {false, false};
    int pipe_par = 0;
    // pipelined pscl_dlscl_device: the baseline's tail (the exact re-decode of its deferred frames,
    // the compaction of the failing frames and their count for the host) runs on tail_stream, so the
    // next call's baseline starts right after this call's screening pass; two parities of deferred-
    // frame scratch (slots 124/125, 126/127) and of count partials (70, 71), ev_tail[q] marks the end of
    // parity q's tail
    hipStream_t tail_stream = nullptr;
    hipEvent_t ev_tscr[2] = {nullptr, nullptr}, ev_tail[2] = {nullptr, nullptr};
    bool tail_pending[2] = {false, false};
    // pipelined pscl_dlscl_device: a call's retry chains (and its DL counters) stay on the retry
    // streams and overlap the next call's baseline decode; the calls alternate the compaction
    // parity (act/cnt), ev_dl[p] marks the end of parity p's chains
    hipEvent_t ev_dl[kDlPar] = {};
    bool dl_pending[kDlPar] = {};
    int dl_par = 0;
    // how many calls back a pipelined call's own buffers may still be in use: for the caller's
    // buffers the depth of pscl_set_pipelined (2 by default: free again at the second following
    // call), kDlPar for pscl_simulate_device's own scratch sets
    int dl_back = 2;
    pscl_dl_call dl_defer;            // the last pipelined call, its chains not yet enqueued
    bool dl_defer_valid = false;
    std::vector<hipEvent_t> ev_pool;
    std::vector<uint8_t> ev_main;     // per timed launch: 1 if it ran on the handle's stream
    size_t ev_used = 0;
    int64_t tune[PSCL_TUNE_COUNT] = {};  // pscl_set_tuning knobs (0 = the default schedule)
    double host_call_ms = 0.0, host_wait_ms = 0.0;  // pscl_host_stats
    int64_t host_calls = 0;
    int64_t n_fpost_rounds = 0, n_post_rounds = 0, n_fused_tx = 0, n_post_epw4 = 0, n_lane_exact = 0;  // pscl_path_stats
};

namespace {

void quiesce(pscl_handle* h);

int ensure(pscl_handle* h, int slot, size_t bytes, void** out) {
    DevBuf& b = h->scratch[slot];
    if (b.n < bytes) {
        if (b.p) {
            quiesce(h);  // (pipelined work may still read it)
            hipFree(b.p);
        }
        b.p = nullptr;
        b.n = 0;
        size_t want = bytes + bytes / 2;  // geometric growth: varying batch sizes settle quickly
        if (want < 4096) want = 4096;
        HIP_TRY(hipMalloc(&b.p, want));
        b.n = want;
    }
    *out = b.p;
    return PSCL_OK;
}

int set_device(pscl_handle* h) {
    HIP_TRY(hipSetDevice(h->device));
    return PSCL_OK;
}

// the handle's stream waits for the pending pipelined work (no host wait): what = 1 the plain
// decodes' re-decodes, 2 the DL-SCL retry chains, 3 both
int dl_enqueue_deferred(pscl_handle* h, bool beside = false);

int join_pipe(pscl_handle* h, int what = 3) {
    if (what & 2) {  // a pipelined DL-SCL call's chains, enqueued first
        const int rc = dl_enqueue_deferred(h);
        if (rc) return rc;
    }
    for (int p = 0; p < 2; ++p)
        if ((what & 2) && h->tail_pending[p]) {
            HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_tail[p], 0));
            h->tail_pending[p] = false;
        }
    for (int p = 0; p < kDlPar; ++p) {
        if ((what & 1) && p < 2 && h->px_pending[p]) {
            HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_px[p], 0));
            h->px_pending[p] = false;
        }
        if ((what & 2) && h->dl_pending[p]) {
            HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_dl[p], 0));
            h->dl_pending[p] = false;
        }
    }
    return PSCL_OK;
}

// every stream the handle's pipelined work may still run on, drained (before a scratch buffer is
// freed and regrown)
void quiesce(pscl_handle* h) {
    if (h->pipe_stream) hipStreamSynchronize(h->pipe_stream);
    if (h->tail_stream) hipStreamSynchronize(h->tail_stream);
    for (int i = 0; i < kChainStreams; ++i) {
        if (h->retry_stream[i]) hipStreamSynchronize(h->retry_stream[i]);
        if (h->side_stream[i]) hipStreamSynchronize(h->side_stream[i]);
    }
}

// destroy the side streams (after draining them) so the next use creates them with the priority
// the handle's current mode asks for (create_priority_stream)
void drop_side_streams(pscl_handle* h) {
    quiesce(h);
    if (h->stash_pipe) hipStreamDestroy(h->stash_pipe);
    h->stash_pipe = nullptr;
    for (int i = 0; i < kChainStreams; ++i) {
        if (h->stash_retry[i]) hipStreamDestroy(h->stash_retry[i]);
        if (h->stash_side[i]) hipStreamDestroy(h->stash_side[i]);
        h->stash_retry[i] = h->stash_side[i] = nullptr;
    }
    if (h->pipe_stream) hipStreamDestroy(h->pipe_stream);
    h->pipe_stream = nullptr;
    if (h->tail_stream) hipStreamDestroy(h->tail_stream);
    h->tail_stream = nullptr;
    for (int i = 0; i < kChainStreams; ++i) {
        if (h->retry_stream[i]) hipStreamDestroy(h->retry_stream[i]);
        if (h->side_stream[i]) hipStreamDestroy(h->side_stream[i]);
        h->retry_stream[i] = h->side_stream[i] = nullptr;
    }
}

// a side stream; on a pipelined handle of the highest priority: latency-bound chains (retry
// rounds, deferred re-decodes) take workgroup slots ahead of the next call's throughput-bound
// baseline decode (measured, config 4 pipelined: 3.55 ms against 4.0 at equal priority).  Not
// otherwise: the FER sweep's two concurrent handles lose from it (4.0 dB point 16.6 -> 25.8 ms)
hipError_t create_priority_stream(pscl_handle* h, hipStream_t* s) {
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) greatest = least = 0;
    const bool plain = h->tune[PSCL_TUNE_SIDE_PRIORITY] == 1;  // (tuning knob: normal priority)
    return hipStreamCreateWithPriority(s, hipStreamNonBlocking, h->pipelined && !plain ? greatest : least);
}

// entry points other than a pipelined plain decode: device, then the pending re-decodes
int enter(pscl_handle* h) {
    const int rc = set_device(h);
    return rc ? rc : join_pipe(h);
}

void fill_decode_params(const pscl_handle* h, pscl_decode_params& P, int hist) {
    memset(&P, 0, sizeof(P));
    P.N = h->N;
    P.n = h->n;
    P.K = h->K;
    P.L = h->L;
    P.W = h->W;
    P.info_mask[0] = h->info_mask[0];
    P.info_mask[1] = h->info_mask[1];
    P.info_words = h->d_info_words;
    P.crc_cols = h->d_check_cols;
    P.info_set = h->d_info_set;
    P.has_crc = h->crc_poly != 0;
    P.exp_table = h->d_exp_table;
    P.epi_table = h->d_epi;
    P.epi_words = h->epi_words;
    P.rm_E = h->rm_E;
    P.rm_src = h->d_rm_src;
    pscl_decode_layout(P, hist);
}

// a counting decode (P.ref) whose kernel stores per-wavefront counts: their buffer (scratch slot 92,
// or 92 + parity for a pipelined plain decode, whose reduce runs on the side stream after its
// re-decode and is ordered before the buffer's next use by ev_px; every other launch is followed
// on its own stream by its count-reduce launch)
// A (re)allocated buffer is zeroed on the decode's own stream st: a plain hipMemset runs on the null
// stream, which the handle's non-blocking streams do not wait for -- the decode could store (and its
// reduce read) partials before the zeroing lands (an intermittent counter mismatch)
int with_count_slots(pscl_handle* h, pscl_decode_params& P, int hist, int slot, hipStream_t st) {
    P.cpart = nullptr;
    const int64_t slots = pscl_decode_count_slots(P, hist);
    if (slots <= 0) return PSCL_OK;
    void* d;
    const size_t had = h->scratch[slot].n;
    const int rc = ensure(h, slot, (size_t)slots * 16, &d);
    if (rc) return rc;
    if (h->scratch[slot].n != had) HIP_TRY(hipMemsetAsync(d, 0, h->scratch[slot].n, st));  // (then kept zero by the reduces)
    P.cpart = (int32_t*)d;
    return PSCL_OK;
}

// scr_slot: the scratch buffer of a long-code decode (decodes that may run concurrently on
// different streams need different slots)
// pipe: the caller is a plain pscl_decode_device on a pipelined handle (see pscl_handle)
// exact decodes on the exact lane-per-path instance where it applies (PSCL_TUNE_LANE_EXACT): off by
// default -- these launches are few frames, bound by one wavefront's latency, and one lane per path
// runs each path's tree updates serially where the two-lanes-per-path kernel splits them: re-decode
// 169 us against 99 us per 10^6-frame headline step, side-chain rounds 208 against 182 us
// (profiles/r06r_lane_exact_ab.txt)
#ifndef PSCL_LANE_EXACT_DEFAULT
#define PSCL_LANE_EXACT_DEFAULT 0
#endif
bool lane_exact_on(const pscl_handle* h) {
    const int64_t lx = h->tune[PSCL_TUNE_LANE_EXACT];
    return lx == 1 || lx == 3 || (lx == 0 && PSCL_LANE_EXACT_DEFAULT);
}

// tail (a pipelined DL-SCL baseline, tail_par its scratch parity): the re-decode of the deferred
// frames goes to tail after the screening pass, and the call returns; the caller queues the rest of
// the baseline's tail there and marks it with ev_tail[tail_par]
int launch_decode(pscl_handle* h, const pscl_decode_params& P0, int hist, hipStream_t st = nullptr, int scr_slot = 38,
                  bool pipe = false, hipStream_t tail = nullptr, int tail_par = 0) {
    if (!st) st = h->stream;
    pscl_decode_params P = P0;
    if (P.long_mode) {  // global scratch of every workgroup in flight (scl_long.hip)
        void* d_scr;
        const int rc = ensure(h, scr_slot, (size_t)pscl_decode_grid(P) * (size_t)P.long_block_bytes, &d_scr);
        if (rc) return rc;
        P.long_scratch = (unsigned char*)d_scr;
    }
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (h->timing) {
        while (h->ev_pool.size() < h->ev_used + 2) {
            hipEvent_t e;
            HIP_TRY(hipEventCreate(&e));
            h->ev_pool.push_back(e);
        }
        e0 = h->ev_pool[h->ev_used];
        e1 = h->ev_pool[h->ev_used + 1];
        if (h->ev_main.size() < h->ev_pool.size() / 2) h->ev_main.resize(h->ev_pool.size() / 2);
        h->ev_main[h->ev_used / 2] = st == h->stream ? 1 : 0;
        h->ev_used += 2;
        HIP_TRY(hipEventRecord(e0, st));
    }
    // Plain decodes of the compiled-in N = 128 codes (no metrics, candidates, decision LLRs,
    // forced bits or row indirection requested) run as a screening decode plus an exact
    // re-decode of the frames it could not certify; the two launches count as one decode.
    // (long codes: the lane-per-path screening kernel, scl_lane_long.hip, N = 256..1024, L = 4, 8)
    pscl_decode_params T = P;
    T.apx = 1;
    const int64_t lx = h->tune[PSCL_TUNE_LANE_EXACT];  // the exact lane-per-path instance (knob 3: every frame)
    const bool screen = h->screen && lx != 3 && !hist && !P.metrics && !P.cands && !P.force && !P.sc_hard && !P.fidx &&
                        !P.d_count &&
                        (P.fast ? (pscl_screening_available(P) != 0 || pscl_lane_long128_available(T) != 0)
                                : pscl_lane_long_available(T) != 0);
    hipError_t err;
    if (!(screen && pipe)) {
        const int rc = join_pipe(h, 1);
        if (rc) return rc;
    }
    if (screen) {
        void *d_cnt, *d_list;
        int rc;
        // pipelined: parity p's list may still be read by the re-decode two calls back
        const int p = pipe ? h->pipe_par : 0;
        const bool tl = tail && !pipe;
        const int s_cnt = tl ? (tail_par ? 126 : 124) : (p ? 64 : 36), s_list = tl ? (tail_par ? 127 : 125) : (p ? 65 : 37);
        if (tl && h->tail_pending[tail_par]) {  // (the parity's previous tail still reads its list)
            if (h->scratch[s_list].n < (size_t)P.B * 8) HIP_TRY(hipEventSynchronize(h->ev_tail[tail_par]));  // (regrown)
            HIP_TRY(hipStreamWaitEvent(st, h->ev_tail[tail_par], 0));
            h->tail_pending[tail_par] = false;
        }
        if (pipe) {
            if (!h->pipe_stream) {
                HIP_TRY(create_priority_stream(h, &h->pipe_stream));
                for (int i = 0; i < 2; ++i) {
                    HIP_TRY(hipEventCreateWithFlags(&h->ev_pscr[i], hipEventDisableTiming));
                    HIP_TRY(hipEventCreateWithFlags(&h->ev_px[i], hipEventDisableTiming));
                }
            }
            if (h->px_pending[p]) {
                if (h->scratch[s_list].n < (size_t)P.B * 8) HIP_TRY(hipEventSynchronize(h->ev_px[p]));  // (regrown)
                HIP_TRY(hipStreamWaitEvent(st, h->ev_px[p], 0));
                h->px_pending[p] = false;
            }
            h->pipe_par ^= 1;
        }
        if ((rc = ensure(h, s_cnt, 4, &d_cnt))) return rc;
        if ((rc = ensure(h, s_list, (size_t)P.B * 8, &d_list))) return rc;
        HIP_TRY(hipMemsetAsync(d_cnt, 0, 4, st));
        pscl_decode_params S = P;
        S.apx = 1;
        pscl_decode_layout(S, hist);  // (no exp table in LDS)
        S.amb_list = (int64_t*)d_list;
        S.amb_count = (int32_t*)d_cnt;
        // (pipelined: the count buffers alternate with the call parity, and the reduce runs on the
        // side stream after the re-decode, off the handle's stream)
        if ((rc = with_count_slots(h, S, hist, tl ? 70 + tail_par : (pipe ? 92 + p : 92), st))) return rc;
        S.tx_upart = nullptr;
        if (S.tx && S.tx_unc_counters) {  // fused TX: the uncoded baseline's per-wavefront partials
            const int64_t slots = pscl_decode_count_slots(S, hist);
            void* du;
            const size_t had = h->scratch[94].n;
            if ((rc = ensure(h, 94, (size_t)(slots > 0 ? slots : 1) * 16, &du))) return rc;
            if (h->scratch[94].n != had) HIP_TRY(hipMemsetAsync(du, 0, h->scratch[94].n, st));  // (then kept zero by the reduces)
            S.tx_upart = (int32_t*)du;
        }
        err = pscl_launch_decode(S, hist, st);
        if (err == hipSuccess && S.tx_upart)
            err = pscl_launch_count_reduce(S.tx_upart, pscl_decode_count_slots(S, hist), S.tx_unc_counters, st);
        if (err == hipSuccess && S.tx)  // fused TX: the deferred frames' rows, read by the exact re-decode
            err = pscl_launch_tx_rows(S, (const int64_t*)d_list, (const int32_t*)d_cnt, S.B, S.tx_rows, S.tx_frame0, st);
        h->screened = true;
        h->screened_slot = s_cnt;
#ifdef PSCL_APX_ABLATE
        // PSCL_DIAG_SCREEN_ONLY=1: timing diagnostics of the screening pass alone (variant
        // builds only, tools/build_variant.py -DPSCL_APX_ABLATE=..); deferred frames stay undecoded
        static const bool screen_only = getenv("PSCL_DIAG_SCREEN_ONLY") && atoi(getenv("PSCL_DIAG_SCREEN_ONLY")) == 1;
#else
        constexpr bool screen_only = false;  // the shipped library always re-decodes deferred frames
#endif
        if (err == hipSuccess && S.cpart && ((!pipe && !tl) || screen_only))
            err = pscl_launch_count_reduce(S.cpart, pscl_decode_count_slots(S, hist), S.counters, st);
        if (err == hipSuccess && !screen_only) {
            pscl_decode_params X = P;  // exact decode of the listed frames, outputs at their rows
            X.tx = 0;                  // (its rows are in HBM: loaded, or written by tx_rows_kernel)
            X.fidx = (const int64_t*)d_list;
            X.d_count = (const int32_t*)d_cnt;
            X.out_by_row = 1;
            X.lane_exact = lane_exact_on(h) ? 1 : 0;
            // few frames: one resident set of workgroups (4 waves/SIMD on 256 CUs), striding
            // over the listed frames, instead of a grid sized for the whole batch
            X.grid_cap = (int64_t)256 * 16 / (pscl_decode_wpg(X) > 0 ? pscl_decode_wpg(X) : 1);
            if (tl) {  // (the caller's tail stream: this call's baseline tail, off the handle's stream)
                if (h->timing) HIP_TRY(hipEventRecord(e1, st));
                HIP_TRY(hipEventRecord(h->ev_tscr[tail_par], st));
                HIP_TRY(hipStreamWaitEvent(tail, h->ev_tscr[tail_par], 0));
                if (!hist && pscl_lane_exact_available(X)) h->n_lane_exact++;
                err = pscl_launch_decode(X, hist, tail);
                if (err == hipSuccess && S.cpart)  // (the screening's count partials, parity slot 70 + tail_par)
                    err = pscl_launch_count_reduce(S.cpart, pscl_decode_count_slots(S, hist), S.counters, tail);
                if (err != hipSuccess) return fail(PSCL_EDEVICE, "decode kernel launch: %s", hipGetErrorString(err));
                return PSCL_OK;
            }
            if (pipe) {
                // the re-decode overlaps the caller's next decode; the timed interval is the
                // screening launch alone
                if (h->timing) HIP_TRY(hipEventRecord(e1, st));
                HIP_TRY(hipEventRecord(h->ev_pscr[p], st));
                HIP_TRY(hipStreamWaitEvent(h->pipe_stream, h->ev_pscr[p], 0));
                if (!hist && pscl_lane_exact_available(X)) h->n_lane_exact++;
                err = pscl_launch_decode(X, hist, h->pipe_stream);
                if (err == hipSuccess && S.cpart)
                    err = pscl_launch_count_reduce(S.cpart, pscl_decode_count_slots(S, hist), S.counters, h->pipe_stream);
                if (err != hipSuccess) return fail(PSCL_EDEVICE, "decode kernel launch: %s", hipGetErrorString(err));
                HIP_TRY(hipEventRecord(h->ev_px[p], h->pipe_stream));
                h->px_pending[p] = true;
                return PSCL_OK;
            }
            if (!hist && pscl_lane_exact_available(X)) h->n_lane_exact++;
            err = pscl_launch_decode(X, hist, st);
        }
    } else {
        if (lx == 3) P.lane_exact = 1;  // (test knob: plain decodes on the exact lane instance)
        const int rc = with_count_slots(h, P, hist, 92, st);
        if (rc) return rc;
        if (!hist && pscl_lane_exact_available(P)) h->n_lane_exact++;
        err = pscl_launch_decode(P, hist, st);
        if (err == hipSuccess && P.cpart) err = pscl_launch_count_reduce(P.cpart, pscl_decode_count_slots(P, hist), P.counters, st);
        if (err == hipSuccess && tail && !pipe) {  // (no screening pass: the caller's tail follows the decode)
            HIP_TRY(hipEventRecord(h->ev_tscr[tail_par], st));
            HIP_TRY(hipStreamWaitEvent(tail, h->ev_tscr[tail_par], 0));
        }
    }
    if (err != hipSuccess) return fail(PSCL_EDEVICE, "decode kernel launch: %s", hipGetErrorString(err));
    if (h->timing) HIP_TRY(hipEventRecord(e1, st));
    return PSCL_OK;
}

}  // namespace

extern "C" {

const char* pscl_last_error(void) { return g_err.c_str(); }

int pscl_abi_version(void) { return PSCL_ABI_VERSION; }

const char* pscl_build_hash(void) { return kBuildHash + 16; }

int pscl_device_count(void) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e == hipErrorNoDevice) return 0;
    if (e != hipSuccess) return fail(PSCL_EDEVICE, "hipGetDeviceCount: %s", hipGetErrorString(e));
    return n;
}

int pscl_create(pscl_handle** out, int device, int N, const int32_t* info_set, int K, int L, uint64_t crc_poly) {
    if (!out) return fail(PSCL_EINVAL, "out is NULL");
    *out = nullptr;
    if (N <= 1 || (N & (N - 1))) return fail(PSCL_EINVAL, "Channel LLR length must be a power of two");
    if (N > PSCL_MAX_N) return fail(PSCL_EUNSUP, "N=%d exceeds PSCL_MAX_N=%d", N, PSCL_MAX_N);
    if (L <= 0) return fail(PSCL_EINVAL, "List size M must be positive");
    if (L > PSCL_MAX_L) return fail(PSCL_EUNSUP, "list size %d exceeds PSCL_MAX_L=%d", L, PSCL_MAX_L);
    if (K < 0 || K > N || (K > 0 && !info_set)) return fail(PSCL_EINVAL, "info_set must hold 0..N indices");
    pscl_handle tmp;
    tmp.N = N;
    while ((1 << tmp.n) < N) tmp.n++;
    tmp.K = K;
    tmp.L = L;
    tmp.W = K > 64 ? (K + 63) / 64 : 1;
    tmp.crc_poly = crc_poly;
    tmp.info_words.assign((size_t)(N >= 64 ? N / 64 : 1), 0ULL);
    for (int i = 0; i < K; ++i) {
        int p = info_set[i];
        if (p < 0 || p >= N) return fail(PSCL_EINVAL, "info_set indices out of range");
        uint64_t bit = 1ULL << (p & 63);
        if (tmp.info_words[(size_t)(p >> 6)] & bit) return fail(PSCL_EUNSUP, "duplicate info_set index %d", p);
        tmp.info_words[(size_t)(p >> 6)] |= bit;
        if (p < PSCL_FAST_N) tmp.info_mask[p >> 6] |= bit;
        tmp.info_set.push_back(p);
    }
    // The decoder visits info phases in increasing phase order; candidate bit j belongs to
    // info_set[j] (u[info_set], scl.py:183).  Both orders agree only for sorted info sets.
    for (int i = 1; i < K; ++i)
        if (tmp.info_set[i] < tmp.info_set[i - 1]) return fail(PSCL_EUNSUP, "info_set must be sorted ascending");
    tmp.check_cols.assign((size_t)(K > 0 ? K : 1), 0u);
    if (crc_poly) {
        tmp.crc_deg = poly_degree(crc_poly);
        if (tmp.crc_deg <= 0) return fail(PSCL_EINVAL, "Polynomial degree must be positive");
        if (tmp.crc_deg > PSCL_MAX_CRC) return fail(PSCL_EUNSUP, "CRC degree %d > %d", tmp.crc_deg, PSCL_MAX_CRC);
        if (K <= tmp.crc_deg) return fail(PSCL_EINVAL, "Message too short for the provided CRC polynomial");
        for (int jj = 0; jj < K; ++jj) {
            std::vector<uint8_t> e((size_t)K, 0);
            e[(size_t)jj] = 1;
            tmp.check_cols[(size_t)jj] = crc_remainder(e, crc_poly, tmp.crc_deg);
        }
        const int kp = K - tmp.crc_deg;
        tmp.attach_cols.assign((size_t)(kp > 0 ? kp : 1), 0u);
        for (int jj = 0; jj < kp; ++jj) {
            std::vector<uint8_t> e((size_t)(kp + tmp.crc_deg), 0);
            e[(size_t)jj] = 1;
            tmp.attach_cols[(size_t)jj] = crc_remainder(e, crc_poly, tmp.crc_deg);
        }
    } else {
        tmp.attach_cols.assign((size_t)(K > 0 ? K : 1), 0u);
    }
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev == 0)
        return fail(PSCL_EDEVICE, "no HIP device available (%s)", e == hipSuccess ? "0 devices" : hipGetErrorString(e));
    if (device < 0 || device >= ndev) return fail(PSCL_EINVAL, "device %d out of range (%d devices)", device, ndev);
    pscl_handle* h = new pscl_handle(tmp);
    h->device = device;
    int rc = set_device(h);
    if (rc) {
        delete h;
        return rc;
    }
#define CREATE_TRY(expr)                                                         \
    do {                                                                         \
        hipError_t _e = (expr);                                                  \
        if (_e != hipSuccess) {                                                  \
            int _c = fail(PSCL_EDEVICE, "%s: %s", #expr, hipGetErrorString(_e)); \
            pscl_destroy(h);                                                     \
            return _c;                                                           \
        }                                                                        \
    } while (0)
    CREATE_TRY(hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking));
    h->stream = h->own_stream;
    CREATE_TRY(hipMalloc(&h->d_check_cols, h->check_cols.size() * 4));
    CREATE_TRY(hipMalloc(&h->d_attach_cols, h->attach_cols.size() * 4));
    CREATE_TRY(hipMalloc(&h->d_info_set, (size_t)(K > 0 ? K : 1) * 4));
    CREATE_TRY(hipMalloc(&h->d_exp_table, sizeof(kExpTable)));
    CREATE_TRY(hipMalloc(&h->d_info_words, h->info_words.size() * 8));
    CREATE_TRY(hipMemcpy(h->d_info_words, h->info_words.data(), h->info_words.size() * 8, hipMemcpyHostToDevice));
    CREATE_TRY(hipMemcpy(h->d_check_cols, h->check_cols.data(), h->check_cols.size() * 4, hipMemcpyHostToDevice));
    CREATE_TRY(hipMemcpy(h->d_attach_cols, h->attach_cols.data(), h->attach_cols.size() * 4, hipMemcpyHostToDevice));
    if (K > 0) CREATE_TRY(hipMemcpy(h->d_info_set, h->info_set.data(), (size_t)K * 4, hipMemcpyHostToDevice));
    CREATE_TRY(hipMemcpy(h->d_exp_table, kExpTable, sizeof(kExpTable), hipMemcpyHostToDevice));
    {
        // NR sub-block interleaver tables (interleaver.py:10-37: order[k] = (k % 32) nb + k / 32 over
        // nb * 32 positions, the identity when N < 32) -- a function of N alone, so they are uploaded
        // here once; pscl_set_rate_match only switches rate matching on or off (no device write
        // while pipelined work may be reading them)
        std::vector<int32_t> order((size_t)N), src((size_t)N);
        const int nb = (N + 31) / 32;
        for (int k = 0; k < N; ++k) order[(size_t)k] = N >= 32 ? (k % 32) * nb + k / 32 : k;
        for (int k = 0; k < N; ++k) src[(size_t)order[(size_t)k]] = k;
        CREATE_TRY(hipMalloc(&h->d_rm_src, (size_t)N * 4));
        CREATE_TRY(hipMalloc(&h->d_rm_order, (size_t)N * 4));
        CREATE_TRY(hipMemcpy(h->d_rm_src, src.data(), (size_t)N * 4, hipMemcpyHostToDevice));
        CREATE_TRY(hipMemcpy(h->d_rm_order, order.data(), (size_t)N * 4, hipMemcpyHostToDevice));
    }
    {
        // scl128 epilogue: gather[k][v] = the information bits of u-byte k (value v), compacted
        // in index order; syn[m][v] = XOR of the CRC check columns of info bits 4m..4m+3 set in v
        // (N > 128: N / 8 gather tables, scl_lane_long.hip)
        const int k4 = (K + 3) / 4, nby = N > 128 ? N / 8 : 16;
        std::vector<uint8_t> epi((size_t)nby * 256 + (size_t)k4 * 16 * 4, 0);
        for (int k = 0; k < nby; ++k)
            for (int v = 0; v < 256; ++v) {
                int c = 0, cntb = 0;
                for (int t = 0; t < 8; ++t) {
                    const int p = 8 * k + t;
                    if (p < N && ((h->info_words[p >> 6] >> (p & 63)) & 1ULL)) {
                        if ((v >> t) & 1) c |= 1 << cntb;
                        cntb++;
                    }
                }
                epi[(size_t)k * 256 + v] = (uint8_t)c;
            }
        uint32_t* syn = reinterpret_cast<uint32_t*>(epi.data() + (size_t)nby * 256);
        for (int m = 0; m < k4; ++m)
            for (int v = 0; v < 16; ++v) {
                uint32_t acc = 0;
                for (int t = 0; t < 4; ++t)
                    if (4 * m + t < K && ((v >> t) & 1)) acc ^= h->check_cols[(size_t)(4 * m + t)];
                syn[m * 16 + v] = acc;
            }
        epi.resize((epi.size() + 7) & ~(size_t)7, 0);
        h->epi_words = (int)(epi.size() / 8);
        CREATE_TRY(hipMalloc(&h->d_epi, epi.size()));
        CREATE_TRY(hipMemcpy(h->d_epi, epi.data(), epi.size(), hipMemcpyHostToDevice));
    }
    {
        // TX tables: encode and CRC attach are GF(2)-linear, so byte-wise tables give them in
        // ceil(K/8) (resp. ceil(kp/8)) lookups per frame.  Codeword words per entry: 2 for
        // N <= 128 (channel_kernel), N / 64 for the long codes (channel_long_kernel).
        const int nb = (K + 7) / 8, kp = K - h->crc_deg, nbp = (kp + 7) / 8;
        const int XW = N <= PSCL_FAST_N ? 2 : N / 64;
        std::vector<uint64_t> xt((size_t)(nb > 0 ? nb : 1) * 256 * XW, 0);
        std::vector<uint64_t> u(XW);
        for (int k = 0; k < nb; ++k)
            for (int v = 0; v < 256; ++v) {
                std::fill(u.begin(), u.end(), 0ULL);
                for (int t = 0; t < 8; ++t) {
                    const int q = 8 * k + t;
                    if (q < K && ((v >> t) & 1)) {
                        const int pos = h->info_set[(size_t)q];
                        u[pos >> 6] |= 1ULL << (pos & 63);
                    }
                }
                for (int w = 0; w < XW; ++w)  // in-word Arikan stages (polar.py:17-29)
                    for (int st = 1; st < 64; st <<= 1) {
                        uint64_t m = 0;
                        for (int b = 0; b < 64; ++b)
                            if (!(b & st)) m |= 1ULL << b;
                        u[w] ^= (u[w] >> st) & m;
                    }
                for (int sw = 1; 64 * sw < N; sw <<= 1)  // stages of 64 bits and more: whole words
                    for (int w = 0; w < XW; ++w)
                        if (!(w & sw) && w + sw < XW) u[w] ^= u[w + sw];
                for (int w = 0; w < XW; ++w) xt[((size_t)k * 256 + v) * XW + w] = u[w];
            }
        std::vector<uint32_t> ct((size_t)(nbp > 0 ? nbp : 1) * 256, 0);
        for (int k = 0; k < nbp; ++k)
            for (int v = 0; v < 256; ++v) {
                uint32_t r = 0;
                for (int t = 0; t < 8; ++t)
                    if (8 * k + t < kp && ((v >> t) & 1)) r ^= h->attach_cols[(size_t)(8 * k + t)];
                ct[(size_t)k * 256 + v] = r;
            }
        CREATE_TRY(hipMalloc(&h->d_xtab, xt.size() * 8));
        CREATE_TRY(hipMemcpy(h->d_xtab, xt.data(), xt.size() * 8, hipMemcpyHostToDevice));
        CREATE_TRY(hipMalloc(&h->d_crctab, ct.size() * 4));
        CREATE_TRY(hipMemcpy(h->d_crctab, ct.data(), ct.size() * 4, hipMemcpyHostToDevice));
    }
#undef CREATE_TRY
    *out = h;
    return PSCL_OK;
}

int pscl_destroy(pscl_handle* h) {
    if (!h) return PSCL_OK;
    hipSetDevice(h->device);
    if (h->dl_defer_valid) dl_enqueue_deferred(h);  // (a pipelined call's chains complete before the buffers go)
    quiesce(h);
    if (h->own_stream) hipStreamSynchronize(h->own_stream);
    if (h->pipe_stream) hipStreamSynchronize(h->pipe_stream);
    for (auto& b : h->scratch)
        if (b.p) hipFree(b.p);
    for (auto e : h->ev_pool) hipEventDestroy(e);
    if (h->d_check_cols) hipFree(h->d_check_cols);
    if (h->d_attach_cols) hipFree(h->d_attach_cols);
    if (h->d_info_set) hipFree(h->d_info_set);
    if (h->d_exp_table) hipFree(h->d_exp_table);
    if (h->d_info_words) hipFree(h->d_info_words);
    if (h->d_rm_src) hipFree(h->d_rm_src);
    if (h->d_rm_order) hipFree(h->d_rm_order);
    if (h->d_beta) hipFree(h->d_beta);
    for (int i = 0; i < 2; ++i)
        if (h->d_beta32g[i]) hipFree(h->d_beta32g[i]);
    if (h->d_epi) hipFree(h->d_epi);
    if (h->d_xtab) hipFree(h->d_xtab);
    if (h->d_crctab) hipFree(h->d_crctab);
    for (int i = 0; i < kChainStreams; ++i)
        if (h->retry_stream[i]) hipStreamSynchronize(h->retry_stream[i]);
    for (int i = 0; i < kDlPar; ++i) {
        if (h->ev_base[i]) hipEventDestroy(h->ev_base[i]);
        if (h->ev_retry[i]) hipEventDestroy(h->ev_retry[i]);
        if (h->ev_dl[i]) hipEventDestroy(h->ev_dl[i]);
    }
    for (int i = 0; i < kChainSets; ++i)
        if (h->ev_join[i]) hipEventDestroy(h->ev_join[i]);
    if (h->h_count) hipHostFree(h->h_count);
    for (int i = 0; i < kChainStreams; ++i) {
        if (h->side_stream[i]) hipStreamSynchronize(h->side_stream[i]);
        if (h->retry_stream[i]) hipStreamDestroy(h->retry_stream[i]);
        if (h->side_stream[i]) hipStreamDestroy(h->side_stream[i]);
        if (h->ev_scr[i]) hipEventDestroy(h->ev_scr[i]);
        if (h->ev_def[i]) hipEventDestroy(h->ev_def[i]);
    }
    for (int i = 0; i < 2; ++i) {
        if (h->ev_pscr[i]) hipEventDestroy(h->ev_pscr[i]);
        if (h->ev_px[i]) hipEventDestroy(h->ev_px[i]);
        if (h->ev_tscr[i]) hipEventDestroy(h->ev_tscr[i]);
        if (h->ev_tail[i]) hipEventDestroy(h->ev_tail[i]);
    }
    if (h->pipe_stream) hipStreamDestroy(h->pipe_stream);
    if (h->tail_stream) hipStreamDestroy(h->tail_stream);
    if (h->stash_pipe) hipStreamDestroy(h->stash_pipe);
    for (int i = 0; i < kChainStreams; ++i) {
        if (h->stash_retry[i]) hipStreamDestroy(h->stash_retry[i]);
        if (h->stash_side[i]) hipStreamDestroy(h->stash_side[i]);
    }
    if (h->own_stream) hipStreamDestroy(h->own_stream);
    delete h;
    return PSCL_OK;
}

int pscl_set_stream(pscl_handle* h, void* s) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    int rc = join_pipe(h);  // pending re-decodes ordered before the old stream's later work
    if (rc) return rc;
    h->stream = s ? (hipStream_t)s : h->own_stream;
    return PSCL_OK;
}

void* pscl_get_stream(pscl_handle* h) { return h ? (void*)h->stream : nullptr; }

int pscl_sync(pscl_handle* h) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    HIP_TRY(hipSetDevice(h->device));
    int rc = join_pipe(h);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(h->stream));
    return PSCL_OK;
}

int pscl_decode_device(pscl_handle* h, const double* d_llr, int64_t B, const uint64_t* d_force, uint64_t* d_best,
                       uint8_t* d_flags, double* d_metrics, uint64_t* d_cands, double* d_info_llrs,
                       const uint64_t* d_ref, int k_payload, int64_t* d_counters) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    if (B < 0) return fail(PSCL_EINVAL, "B must be >= 0");
    if (B == 0) return PSCL_OK;
    if (!d_llr) return fail(PSCL_EINVAL, "d_llr is NULL");
    if (d_ref && !d_counters) return fail(PSCL_EINVAL, "d_ref given without d_counters");
    if (k_payload < 0 || k_payload > h->K) return fail(PSCL_EINVAL, "k_payload out of range");
    int rc = set_device(h);
    if (rc) return rc;
    const int hist = d_info_llrs != nullptr;
    pscl_decode_params P;
    fill_decode_params(h, P, hist);
    P.llr = d_llr;
    P.B = B;
    P.force = d_force;
    P.best = d_best;
    P.flags = d_flags;
    P.metrics = d_metrics;
    P.cands = d_cands;
    P.info_llrs = d_info_llrs;
    P.ref = d_ref;
    P.k_payload = k_payload;
    P.counters = d_counters;
    if (pscl_decode_wpg(P) < 1) return fail(PSCL_EUNSUP, "LDS budget exceeded (L=%d, K=%d)", h->L, h->K);
    if (!h->pipelined && (rc = join_pipe(h))) return rc;
    return launch_decode(h, P, hist, nullptr, 38, h->pipelined);
}

int pscl_join(pscl_handle* h) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    int rc = set_device(h);
    if (rc) return rc;
    return join_pipe(h);
}

int pscl_set_pipelined(pscl_handle* h, int enable) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    int rc = set_device(h);
    if (rc) return rc;
    if ((rc = join_pipe(h))) return rc;
    if (enable < 0 || enable > kDlPar) return fail(PSCL_EINVAL, "pipelined depth %d out of range 0..%d", enable, kDlPar);
    if (h->pipelined != (enable != 0)) {
        // the other mode's streams in, this mode's to the stash (drained first)
        quiesce(h);
        std::swap(h->pipe_stream, h->stash_pipe);
        for (int i = 0; i < kChainStreams; ++i) {
            std::swap(h->retry_stream[i], h->stash_retry[i]);
            std::swap(h->side_stream[i], h->stash_side[i]);
        }
    }
    h->pipelined = enable != 0;
    // DL-SCL calls: a call's buffers are free again at the depth-th following call (1 and 2: the
    // second, the documented default); its chains run up to depth - 1 calls behind the baselines
    h->dl_back = enable >= 2 ? enable : 2;
    return PSCL_OK;
}

int pscl_set_tuning(pscl_handle* h, int knob, int64_t value) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    static const int64_t lim[PSCL_TUNE_COUNT][2] = {{0, 0}, {0, 2}, {0, 64}, {0, 2}, {0, 1}, {0, 4096}, {0, PSCL_MAX_WAVES_PER_WG}, {0, 2},
                                                    {0, (int64_t)1 << 30}, {0, 2}, {0, 32}, {0, 3}, {0, 2}, {0, 2}, {0, 4}, {0, 3}, {0, 2}, {0, 1}};
    if (knob < 1 || knob >= PSCL_TUNE_COUNT) return fail(PSCL_EINVAL, "unknown tuning knob %d", knob);
    if (value < lim[knob][0] || value > lim[knob][1] || (knob == PSCL_TUNE_POST_GRID && value && value < 16))
        return fail(PSCL_EINVAL, "tuning knob %d: value %lld out of range", knob, (long long)value);
    if (knob == PSCL_TUNE_POST_EPW && value != 0 && value != 2 && value != 4)
        return fail(PSCL_EINVAL, "tuning knob %d: value %lld out of range", knob, (long long)value);
    int rc = set_device(h);
    if (rc) return rc;
    if ((rc = join_pipe(h))) return rc;  // (pending work ran under the old schedule)
    if (knob == PSCL_TUNE_SIDE_PRIORITY && h->tune[knob] != value) drop_side_streams(h);
    h->tune[knob] = value;
    return PSCL_OK;
}

int pscl_path_llrs_device(pscl_handle* h, const double* d_llr, int64_t B, const uint64_t* d_bits, double* d_out) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    if (B < 0) return fail(PSCL_EINVAL, "B must be >= 0");
    if (B == 0) return PSCL_OK;
    if (!d_llr || !d_bits || !d_out) return fail(PSCL_EINVAL, "d_llr, d_bits and d_out are required");
    if (h->N > PSCL_FAST_N) return fail(PSCL_EUNSUP, "decision-LLR replay supports N <= %d", PSCL_FAST_N);
    if (B > INT32_MAX) return fail(PSCL_EUNSUP, "B exceeds 2^31-1");
    int rc = enter(h);
    if (rc) return rc;
    void *d_cnt, *d_rows;
    if ((rc = ensure(h, 25, 8, &d_cnt))) return rc;
    if ((rc = ensure(h, 26, (size_t)B * 8, &d_rows))) return rc;
    const int32_t nb = (int32_t)B;
    HIP_TRY(hipMemcpyAsync(d_cnt, &nb, 4, hipMemcpyHostToDevice, h->stream));
    hipError_t e = pscl_launch_iota64((int64_t*)d_rows, B, h->stream);
    if (e != hipSuccess) return fail(PSCL_EDEVICE, "iota launch: %s", hipGetErrorString(e));
    pscl_replay_params Rp;
    memset(&Rp, 0, sizeof(Rp));
    Rp.llr = d_llr;
    Rp.N = h->N;
    Rp.n = h->n;
    Rp.K = h->K;
    Rp.W = h->W;
    Rp.rm_E = h->rm_E;
    Rp.rm_src = h->d_rm_src;
    Rp.info_mask[0] = h->info_mask[0];
    Rp.info_mask[1] = h->info_mask[1];
    Rp.count = (const int32_t*)d_cnt;
    Rp.act = (const int64_t*)d_rows;
    Rp.bits = d_bits;
    Rp.bits_by_row = 1;
    Rp.out = d_out;
    if ((e = pscl_launch_replay(Rp, B, h->stream)) != hipSuccess)
        return fail(PSCL_EDEVICE, "replay launch: %s", hipGetErrorString(e));
    HIP_TRY(hipStreamSynchronize(h->stream));  // d_cnt is a host-staged value
    return PSCL_OK;
}

int pscl_set_beta(pscl_handle* h, const double* beta) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    int rc = enter(h);
    if (rc) return rc;
    if (!beta) {
        if (h->d_beta) HIP_TRY(hipFree(h->d_beta));
        h->d_beta = nullptr;
        for (int i = 0; i < 2; ++i) {
            if (h->d_beta32g[i]) HIP_TRY(hipFree(h->d_beta32g[i]));
            h->d_beta32g[i] = nullptr;
        }
        return PSCL_OK;
    }
    if (h->K == 0) return fail(PSCL_EINVAL, "beta must be a square matrix matching abs_l0 length");
    const size_t n = (size_t)h->K * h->K;
    if (!h->d_beta) HIP_TRY(hipMalloc(&h->d_beta, n * 8));
    // stream-ordered upload: enter() made the handle's stream wait for every pending pipelined
    // round (which may still read the old matrix), so the copy lands after them and before any
    // later launch; the host staging buffer is rewritten only once the previous upload is done
    HIP_TRY(hipStreamSynchronize(h->stream));
    h->beta_host.assign(beta, beta + n);
    HIP_TRY(hipMemcpyAsync(h->d_beta, h->beta_host.data(), n * 8, hipMemcpyHostToDevice, h->stream));
    if (h->K == 64) {  // the fused post pass's layouts: lane p's candidates p + G i contiguous per row k
        const int K = h->K;
        h->beta32g_host.assign(2 * n, 0.0f);
        for (int gi = 0; gi < 2; ++gi) {
            const int G = gi ? 4 : 8, NC = K / G;
            for (int k = 0; k < K; ++k)
                for (int pp = 0; pp < G; ++pp)
                    for (int i = 0; i < NC; ++i)
                        h->beta32g_host[(size_t)gi * n + ((size_t)k * G + pp) * NC + i] = (float)beta[(size_t)k * K + pp + G * i];
            if (!h->d_beta32g[gi]) HIP_TRY(hipMalloc(&h->d_beta32g[gi], n * 4));
            HIP_TRY(hipMemcpyAsync(h->d_beta32g[gi], h->beta32g_host.data() + (size_t)gi * n, n * 4, hipMemcpyHostToDevice,
                                   h->stream));
        }
    }
    double mx = 0.0;
    bool nan = false;
    for (size_t i = 0; i < n; ++i) {
        const double a = fabs(beta[i]);
        if (std::isnan(a))
            nan = true;
        else if (a > mx)
            mx = a;
    }
    h->beta_absmax = nan ? INFINITY : mx;  // (a NaN entry: every certificate fails, exact sums)
    return PSCL_OK;
}

// retry rounds of one chunk on the retry stream (state sized for the largest chunk)
#ifndef PSCL_DL_FUSED_POST_DEFAULT
#define PSCL_DL_FUSED_POST_DEFAULT 0
#endif
namespace {
struct DlState {
    int64_t* act;     // [cap] frame index of each entry (a slice of the chunk's dl_compact output)
    int32_t* bcnt;    // [rounds + 1][NSEG * CSTRIDE] bucket counters of each round's list
    int32_t *list0, *list1;  // [NSEG][cap] bucket lists (entry ids), alternating rounds
    uint64_t *tried, *force, *warm_u, *ob;
    int32_t* nt;
    double* warm_metric;
    uint8_t* of;
    int32_t *dcnt, *dlist;   // screening retry decodes: the side chain's bucket lists, one per round
                             // ([rounds + 1][NSEG * CSTRIDE] counts, [rounds + 1][NSEG][cap])
    uint64_t* ob2;           // [cap][W] and [cap]: their exact decode's outputs (the main post pass reads
    uint8_t* of2;            //   `of` concurrently, where the deferred mark must stay)
};

#ifndef PSCL_DL_WARM_APX_DEFAULT
#define PSCL_DL_WARM_APX_DEFAULT 1  // (measured: profiles/r06t_warm_apx_ab.txt)
#endif

hipError_t launch_post(pscl_handle* h, const pscl_post_params& Q, int64_t A, hipStream_t s) {
    if (pscl_post_epw(Q) == 4) h->n_post_epw4++;
    return pscl_launch_dl_post(Q, A, s);
}

int dl_retry_chunk(pscl_handle* h, const DlState& S, int A, int rounds, const double* d_llr, uint64_t* d_best,
                   uint8_t* d_flags, int32_t* d_attempts, int32_t* d_tried, int tried_stride, int64_t* d_cnt_dl,
                   hipStream_t st, hipStream_t side, hipEvent_t ev_s, hipEvent_t ev_d, bool narrow, bool beside) {
    const int K = h->K, W = h->W;
    hipError_t e;
    const size_t bstride = (size_t)PSCL_DL_NSEG * PSCL_DL_CSTRIDE;
    HIP_TRY(hipMemsetAsync(S.bcnt, 0, (size_t)(rounds + 1) * bstride * 4, st));
    pscl_post_params Q;
    memset(&Q, 0, sizeof(Q));
    Q.llr = d_llr;
    Q.N = h->N;
    Q.n = h->n;
    Q.K = K;
    Q.W = W;
    Q.rm_E = h->rm_E;
    Q.rm_src = h->d_rm_src;
    Q.info_mask[0] = h->info_mask[0];
    Q.info_mask[1] = h->info_mask[1];
    Q.info_set = h->d_info_set;
    Q.exp_table = h->d_exp_table;
    Q.rounds = rounds;
    Q.narrow = narrow ? 1 : 0;  // (pipelined calls: beside the next call's baseline)
    Q.grid_cap = h->tune[PSCL_TUNE_POST_GRID];
    Q.pairs = h->tune[PSCL_TUNE_POST_PAIRS];
    Q.epw = (int)h->tune[PSCL_TUNE_POST_EPW];
    Q.cap = A;
    Q.act = S.act;
    Q.tried = S.tried;
    Q.ntried = S.nt;
    Q.beta = h->d_beta;
    Q.beta_absmax = h->beta_absmax;
    Q.force = S.force;
    Q.warm_metric = S.warm_metric;
    Q.warm_u = S.warm_u;
    Q.ob = S.ob;
    Q.of = S.of;
    Q.best = d_best;
    Q.flags = d_flags;
    Q.attempts = d_attempts;
    Q.tried_out = d_tried;
    Q.tried_stride = tried_stride;
    Q.counters = d_cnt_dl;
    int32_t* lists[2] = {S.list0, S.list1};
    // the retry decodes: entries bucket by bucket, LLR rows by indirection, forced prefixes,
    // warm-started past them (the compiled-in FS kernels; others decode from phase 0)
    pscl_decode_params H;
    fill_decode_params(h, H, 0);
    H.llr = d_llr;
    H.B = A;
    H.fidx = S.act;
    H.force = S.force;
    H.best = S.ob;
    H.flags = S.of;
    H.bcap = A;
    H.warm_metric = S.warm_metric;
    H.warm_u = S.warm_u;
    H.wpg_cap = (int)h->tune[PSCL_TUNE_RETRY_WPG];
    H.lane_exact = lane_exact_on(h) ? 1 : 0;  // (exact retry rounds: the lane-per-path instance)
    if (pscl_decode_wpg(H) < 1) return fail(PSCL_EUNSUP, "LDS budget exceeded (L=%d, K=%d)", h->L, h->K);
    int rc;
    // screening retry decodes (measured in DESIGN.md §5.4): the forced-bit screening instance
    // decodes the round's entries and moves the ones it cannot certify to a SIDE CHAIN (flags
    // PSCL_DL_DEFERRED, which the main post pass skips): on the side stream, round r of the side
    // chain decodes its entries exactly (warm-started, as every retry decode) -- the ones round r
    // of the main chain deferred plus the side chain's own survivors -- and its post pass files the
    // survivors in the side chain's list of round r + 1.  An entry stays on the side chain once
    // deferred, at the same attempt index as the main chain's round, so the main chain never waits
    // for the side chain's exact decodes; the chain ends with both.  Each round has its own side
    // list (the side chain may lag the main chain by several rounds).
    // screening retry decodes: always (1), never (2), or by default (0) every chain, unless
    // PSCL_TUNE_DL_SCREEN_MIN sets a size threshold (chains of at least that many entries, and every
    // chain beside a later baseline decode).  With the deferred entries on the side chain the main
    // chain never waits for an exact decode, so screening wins alone too: the standalone config-3
    // 5 dB point (~10^4 entries per round) 4.61-4.62 -> 4.32 ms, the sweep 283.7 -> 285.1 M frames/s
    // (profiles/r05v_screen_ab.txt; round 4, before the side chain, it lost alone: 5.6 -> 6.1 ms)
    const int64_t ds = h->tune[PSCL_TUNE_DL_SCREEN];
    const int64_t ds_min = h->tune[PSCL_TUNE_DL_SCREEN_MIN];
    const bool dl_screen = ds == 1 || (ds == 0 && (!ds_min || A >= ds_min || beside));
    const bool scr = dl_screen && h->screen && S.dcnt && S.ob2 && side && pscl_screening_fs_available(H);
    pscl_decode_params HA, HX;
    pscl_post_params QD;
    bool fpost = false;  // the main chain's post pass inside its screened retry decodes
    if (scr) {
        HA = H;
        HA.apx = 1;
        pscl_decode_layout(HA, 0);  // (no exp table in LDS)
        HA.no_lane = h->tune[PSCL_TUNE_DL_RETRY_LANE] == 2 ? 1 : 0;  // (lane-per-path FS kernel by default)
        const int64_t fk = h->tune[PSCL_TUNE_DL_FUSED_POST];
        pscl_decode_params T = HA;  // (the rounds' launches: bucket lists in and deferred lists out)
        T.elist = lists[0];
        T.bcount = S.bcnt;
        T.amb_elist = S.dlist;
        T.amb_count = S.dcnt;
        fpost = (fk == 1 || (fk == 0 && PSCL_DL_FUSED_POST_DEFAULT)) && !HA.no_lane && pscl_lane_fs_available(T) &&
                h->K == 64 && (!h->d_beta || h->d_beta32g[h->L == 8 ? 0 : 1]);
        if (fpost) {
            HA.fpost = 1;
            HA.fp = Q;
            HA.fp.init = 0;
            HA.fp_beta32g = h->d_beta ? h->d_beta32g[h->L == 8 ? 0 : 1] : nullptr;
        }
        HX = H;
        HX.best = S.ob2;
        HX.flags = S.of2;
        HX.grid_cap = (int64_t)256 * 16 / (pscl_decode_wpg(HX) > 0 ? pscl_decode_wpg(HX) : 1);
        QD = Q;
        QD.init = 0;
        QD.ob = S.ob2;
        QD.of = S.of2;
        HIP_TRY(hipMemsetAsync(S.dcnt, 0, (size_t)(rounds + 1) * bstride * 4, st));
        // the main chain's warm-start metrics from the screening tail (PSCL_TUNE_DL_WARM_APX): its
        // screened decodes certify against margins that cover every increment's tail error, the
        // prefix's too; the entries they defer go to the side chain's bucket 0 (exact from phase 0),
        // whose own posts (QD) keep exact metrics
        // (default: for chains beside a later baseline decode, which are throughput-bound; a chain
        // running alone is latency-bound, and its side chain -- the longer one -- keeps warm starts)
        const int64_t wk = h->tune[PSCL_TUNE_DL_WARM_APX];
        if (!fpost && (wk == 1 || (wk == 0 && PSCL_DL_WARM_APX_DEFAULT && beside))) {
            Q.warm_apx = 1;
            HA.warm_apx = 1;
        }
    }
    // first flips: replay of every baseline best path (flip.py:97-111)
    Q.init = 1;
    Q.in_count = nullptr;
    Q.out_count = S.bcnt;
    Q.out_list = lists[0];
    if ((e = launch_post(h, Q, A, st)) != hipSuccess) return fail(PSCL_EDEVICE, "dl_post launch: %s", hipGetErrorString(e));
    auto side_list = [&](int r) { return S.dlist + (size_t)r * PSCL_DL_NSEG * (size_t)A; };
    auto side_cnt = [&](int r) { return S.dcnt + (size_t)r * bstride; };
    Q.init = 0;
    for (int r = 0; r < rounds; ++r) {  // no host round trips: the counts stay on the device
        H.elist = lists[r & 1];
        H.bcount = S.bcnt + (size_t)r * bstride;
        if (scr) {
            HA.elist = H.elist;
            HA.bcount = H.bcount;
            HA.amb_elist = side_list(r);  // (the side chain's round-r list: appended beside QD(r - 1))
            HA.amb_count = side_cnt(r);
            if (fpost) {  // the round's survivors to the next round's lists, filed by the decode itself
                HA.fp.in_count = H.bcount;
                HA.fp.in_list = lists[r & 1];
                HA.fp.out_count = S.bcnt + (size_t)(r + 1) * bstride;
                HA.fp.out_list = lists[(r + 1) & 1];
            }
            if ((e = pscl_launch_decode(HA, 0, st)) != hipSuccess)
                return fail(PSCL_EDEVICE, "screening retry decode: %s", hipGetErrorString(e));
            HIP_TRY(hipEventRecord(ev_s, st));
            // side round r: after the main round's deferrals (ev_s) and side round r - 1 (stream order)
            HIP_TRY(hipStreamWaitEvent(side, ev_s, 0));
            HX.elist = side_list(r);
            HX.bcount = side_cnt(r);
            if (pscl_lane_exact_available(HX)) h->n_lane_exact++;
            if ((e = pscl_launch_decode(HX, 0, side)) != hipSuccess)
                return fail(PSCL_EDEVICE, "exact retry re-decode: %s", hipGetErrorString(e));
            QD.in_list = side_list(r);
            QD.in_count = side_cnt(r);
            QD.out_list = side_list(r + 1);
            QD.out_count = side_cnt(r + 1);
            if ((e = launch_post(h, QD, A, side)) != hipSuccess)
                return fail(PSCL_EDEVICE, "dl_post launch: %s", hipGetErrorString(e));
        } else if ((rc = launch_decode(h, H, 0, st))) {
            return rc;
        }
        if (fpost) {  // (the decode ran the main chain's post pass)
            h->n_fpost_rounds++;
            continue;
        }
        h->n_post_rounds++;
        Q.in_count = H.bcount;
        Q.in_list = lists[r & 1];
        Q.out_count = S.bcnt + (size_t)(r + 1) * bstride;
        Q.out_list = lists[(r + 1) & 1];
        if ((e = launch_post(h, Q, A, st)) != hipSuccess)
            return fail(PSCL_EDEVICE, "dl_post launch: %s", hipGetErrorString(e));
    }
    if (scr && rounds > 0) {  // the chain ends with its side chain
        HIP_TRY(hipEventRecord(ev_d, side));
        HIP_TRY(hipStreamWaitEvent(st, ev_d, 0));
    }
    return PSCL_OK;
}

// long codes (N > PSCL_FAST_N): dense entry state, ping-ponged between passes; the retry
// decodes' workgroup scratch has its own slot (they may overlap the next chunk's baseline)
constexpr int kLongRetryScratch = 62;
struct DlLongState {
    int64_t* act1;              // the second entry-frame array (the first is the compaction's)
    uint64_t *tried[2], *ob, *force;
    int32_t *nt[2], *cnt;       // cnt: [rounds + 2] entries of each pass
    uint8_t* of;
    double* l0;
};

// The retry chain of a chunk's A failing frames (act0/cnt0: dl_compact's output) for the long
// codes: the failing frames decoded again with decision-LLR history (the baseline's L0,
// flip.py:97-102; same best bits), a first post pass, then per round a HIST decode of the live
// entries (forced bits, LLR rows by indirection, the live count on the device) and a post pass.
int dl_retry_long(pscl_handle* h, const DlLongState& S, int64_t* act0, const int32_t* cnt0, int A, int rounds,
                  const double* d_llr, uint64_t* d_best, uint8_t* d_flags, int32_t* d_attempts, int32_t* d_tried,
                  int tried_stride, int64_t* d_cnt_dl, hipStream_t st) {
    hipError_t e;
    int rc;
    HIP_TRY(hipMemsetAsync(S.cnt, 0, (size_t)(rounds + 2) * 4, st));
    pscl_decode_params H;
    fill_decode_params(h, H, 1);
    H.llr = d_llr;
    H.B = A;
    H.fidx = act0;
    H.d_count = cnt0;
    H.best = S.ob;
    H.flags = S.of;
    H.best_info_llrs = S.l0;
    if ((rc = launch_decode(h, H, 1, st, kLongRetryScratch))) return rc;
    pscl_post_long_params Q;
    memset(&Q, 0, sizeof(Q));
    Q.K = h->K;
    Q.W = h->W;
    Q.rounds = rounds;
    Q.cap = A;
    Q.ob = S.ob;
    Q.of = S.of;
    Q.l0 = S.l0;
    Q.force = S.force;
    Q.beta = h->d_beta;
    Q.best = d_best;
    Q.flags = d_flags;
    Q.attempts = d_attempts;
    Q.tried_out = d_tried;
    Q.tried_stride = tried_stride;
    Q.counters = d_cnt_dl;
    int64_t* acts[2] = {act0, S.act1};
    Q.init = 1;
    Q.in_count = cnt0;
    Q.out_count = S.cnt + 1;
    Q.act_in = act0;
    Q.act_out = S.act1;
    Q.tried_w_out = S.tried[1];
    Q.nt_out = S.nt[1];
    if ((e = pscl_launch_dl_post_long(Q, st)) != hipSuccess)
        return fail(PSCL_EDEVICE, "dl_post_long launch: %s", hipGetErrorString(e));
    Q.init = 0;
    for (int r = 0; r < rounds; ++r) {  // pass r + 1 reads state set (r + 1) & 1
        const int c = (r + 1) & 1;
        H.fidx = acts[c];
        H.d_count = S.cnt + r + 1;
        H.force = S.force;
        if ((rc = launch_decode(h, H, 1, st, kLongRetryScratch))) return rc;
        Q.in_count = S.cnt + r + 1;
        Q.out_count = S.cnt + r + 2;
        Q.act_in = acts[c];
        Q.act_out = acts[c ^ 1];
        Q.tried_in = S.tried[c];
        Q.tried_w_out = S.tried[c ^ 1];
        Q.nt_in = S.nt[c];
        Q.nt_out = S.nt[c ^ 1];
        if ((e = pscl_launch_dl_post_long(Q, st)) != hipSuccess)
            return fail(PSCL_EDEVICE, "dl_post_long launch: %s", hipGetErrorString(e));
    }
    return PSCL_OK;
}
}  // namespace

namespace {
constexpr int kMinSplit = 2048;

// the retry chains' state (scratch slots), sized by dl_setup
struct DlBufs {
    DlState S[kChainStreams];  // chain state (S[2 set + k] on retry stream 2 set + k)
    DlLongState LS = {};  // (long codes)
    int32_t* cnt[kDlPar] = {};  // failing-frame count of the compaction parities
    int64_t* act[kDlPar] = {};  // their frame indices
};

// compaction parity of chunk c: a pipelined call (one chunk) takes the handle's rotating parity,
// the chunks of an unpipelined call alternate two
inline int dl_parity(const pscl_dl_call& a, int64_t c) { return a.pipe ? a.pbase : (int)(c & 1); }
constexpr int kCntSlot[kDlPar] = {22, 27, 80, 82}, kActSlot[kDlPar] = {23, 28, 81, 83};

// streams, events and scratch of a DL-SCL call (everything sized before any work is queued:
// an allocation synchronizes the device)
int dl_setup(pscl_handle* h, const pscl_dl_call& a, DlBufs& b) {
    int rc;
    const int K = h->K, W = h->W, rounds = a.rounds;
    const int64_t cap = a.cap;
    // chain sets: a pipelined call's chains (or an unpipelined call's chunk chains) alternate two
    const int nsets = (h->N <= PSCL_FAST_N && (a.pipe || a.nch >= 2)) ? kChainSets : 1;
    // (only the streams of the chains this call runs: chain i of set s is stream 2 s + i, i < nsplit;
    // every extra stream of the process shifts how the runtime spreads streams over its hardware queues)
    for (int i = 0; i < 2 * nsets; ++i)
        if (!h->retry_stream[i] && (i & 1) < (a.nsplit > 0 ? a.nsplit : 1)) HIP_TRY(create_priority_stream(h, &h->retry_stream[i]));
    for (int i = 0; i < kDlPar; ++i) {
        if (!h->ev_base[i]) HIP_TRY(hipEventCreateWithFlags(&h->ev_base[i], hipEventDisableTiming));
        if (!h->ev_retry[i]) HIP_TRY(hipEventCreateWithFlags(&h->ev_retry[i], hipEventDisableTiming));
        if (!h->ev_dl[i]) HIP_TRY(hipEventCreateWithFlags(&h->ev_dl[i], hipEventDisableTiming));
    }
    for (int i = 0; i < 2 * nsets; ++i) {
        if ((i & 1) >= (a.nsplit > 0 ? a.nsplit : 1)) continue;
        if (!h->side_stream[i]) HIP_TRY(create_priority_stream(h, &h->side_stream[i]));
        if (!h->ev_scr[i]) HIP_TRY(hipEventCreateWithFlags(&h->ev_scr[i], hipEventDisableTiming));
        if (!h->ev_def[i]) HIP_TRY(hipEventCreateWithFlags(&h->ev_def[i], hipEventDisableTiming));
    }
    for (int i = 0; i < nsets; ++i)
        if (!h->ev_join[i]) HIP_TRY(hipEventCreateWithFlags(&h->ev_join[i], hipEventDisableTiming));
    if (!h->h_count) HIP_TRY(hipHostMalloc((void**)&h->h_count, 4 * kDlPar, hipHostMallocDefault));
    const size_t NS = PSCL_DL_NSEG;
    for (int i = 0; i < (a.pipe ? kDlPar : (a.nch >= 2 ? 2 : 1)); ++i) {
        void *pc, *pa;
        if ((rc = ensure(h, kCntSlot[i], 4, &pc)) || (rc = ensure(h, kActSlot[i], (size_t)cap * 8, &pa))) return rc;
        b.cnt[i] = (int32_t*)pc;
        b.act[i] = (int64_t*)pa;
    }
    if (h->N > PSCL_FAST_N) {  // long codes: one chain, dense state (dl_retry_long)
        const size_t c = (size_t)cap;
        const size_t sz[10] = {c * 8, c * W * 8, c * W * 8, c * W * 8, c * 2 * W * 8, c * 4, c * 4,
                               (size_t)(rounds + 2) * 4, c, c * K * 8};
        void* q[10];
        for (int k = 0; k < 10; ++k)
            if ((rc = ensure(h, 52 + k, sz[k], &q[k]))) return rc;
        b.LS.act1 = (int64_t*)q[0];
        b.LS.tried[0] = (uint64_t*)q[1];
        b.LS.tried[1] = (uint64_t*)q[2];
        b.LS.ob = (uint64_t*)q[3];
        b.LS.force = (uint64_t*)q[4];
        b.LS.nt[0] = (int32_t*)q[5];
        b.LS.nt[1] = (int32_t*)q[6];
        b.LS.cnt = (int32_t*)q[7];
        b.LS.of = (uint8_t*)q[8];
        b.LS.l0 = (double*)q[9];
        pscl_decode_params H;  // the retry decodes' scratch
        fill_decode_params(h, H, 1);
        H.B = cap;
        void* d_scr;
        if ((rc = ensure(h, kLongRetryScratch, (size_t)pscl_decode_grid(H) * (size_t)H.long_block_bytes, &d_scr)))
            return rc;
    }
    for (int j = 0; j < 2 * nsets; ++j) {
        // chain 0 takes every entry of a call that does not split (fewer than 2 kMinSplit
        // failing frames, which may still exceed half the chunk); chain 1 at most half
        const int i = j & 1, set = j >> 1;
        if (i >= a.nsplit) continue;
        const size_t c = (size_t)(i == 0 ? cap : cap - cap / 2);
        const size_t sz[14] = {(size_t)(rounds + 1) * NS * PSCL_DL_CSTRIDE * 4, NS * c * 4, NS * c * 4, c * 16, c * 4,
                               c * 2 * W * 8, c * NS * 8, c * 16, c * W * 8, c,
                               (size_t)(rounds + 1) * NS * PSCL_DL_CSTRIDE * 4, (size_t)(rounds + 1) * NS * c * 4,
                               c * W * 8, c};
        static const int slot[kChainStreams][14] = {{12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 8, 9, 10, 11},
                                                    {40, 41, 42, 43, 44, 45, 46, 47, 48, 49, 50, 51, 24, 29},
                                                    {96, 97, 98, 99, 100, 101, 102, 103, 104, 105, 106, 107, 108, 109},
                                                    {110, 111, 112, 113, 114, 115, 116, 117, 118, 119, 120, 121, 122, 123}};
        void* q[14];
        for (int k = 0; k < 14; ++k)
            if ((rc = ensure(h, slot[j][k], sz[k], &q[k]))) return rc;
        DlState& T = b.S[2 * set + i];
        T.dcnt = (int32_t*)q[10];
        T.dlist = (int32_t*)q[11];
        T.ob2 = (uint64_t*)q[12];
        T.of2 = (uint8_t*)q[13];
        T.bcnt = (int32_t*)q[0];
        T.list0 = (int32_t*)q[1];
        T.list1 = (int32_t*)q[2];
        T.tried = (uint64_t*)q[3];
        T.nt = (int32_t*)q[4];
        T.force = (uint64_t*)q[5];
        T.warm_metric = (double*)q[6];
        T.warm_u = (uint64_t*)q[7];
        T.ob = (uint64_t*)q[8];
        T.of = (uint8_t*)q[9];
    }
    return PSCL_OK;
}

// the chain set of chunk c: alternating by call (pipelined) or by chunk; the long codes' single
// dense-state chain keeps set 0
inline int dl_set(const pscl_handle* h, const pscl_dl_call& a, int64_t c) {
    if (h->tune[PSCL_TUNE_DL_STREAMS] & 2) return 0;  // (one set: chains in call order on its streams)
    return h->N > PSCL_FAST_N ? 0 : (a.pipe ? a.pbase : (int)c) & (kChainSets - 1);
}

// the retry chains of chunk c (compaction parity p): the host reads the chunk's failing count
// (waiting for its baseline) and enqueues the rounds on the retry streams of the chunk's set;
// ev_retry[p] marks their end on the set's first retry stream
int dl_chain(pscl_handle* h, const pscl_dl_call& a, const DlBufs& b, int64_t c, bool beside) {
    const int p = dl_parity(a, c);
    const int cs = 2 * dl_set(h, a, c);  // the set's first stream
    const int64_t cap = a.cap;
    const auto w0 = std::chrono::steady_clock::now();
    HIP_TRY(hipEventSynchronize(h->ev_base[p]));
    h->host_wait_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
    const int A = h->h_count[p];
    int64_t* d_cdl = a.d_ref ? a.d_counters_dl : nullptr;
    if (h->N > PSCL_FAST_N) {
        if (A > 0) {
            HIP_TRY(hipStreamWaitEvent(h->retry_stream[0], h->ev_base[p], 0));
            int r2 = dl_retry_long(h, b.LS, b.act[p], b.cnt[p], A, a.rounds, a.d_llr, a.d_best, a.d_flags, a.d_attempts,
                                   a.d_tried, a.tried_stride, d_cdl, h->retry_stream[0]);
            if (r2) return r2;
        }
        HIP_TRY(hipEventRecord(h->ev_retry[p], h->retry_stream[0]));
        return PSCL_OK;
    }
    const int parts = (a.nsplit == 2 && A >= 2 * kMinSplit) ? 2 : 1;
    const int A0 = parts == 2 ? A - A / 2 : A;
    for (int k = 0; k < parts && A > 0; ++k) {
        const int64_t nk = k ? A - A0 : A0, capk = k ? cap - cap / 2 : cap;  // (state sized by dl_setup)
        if (nk > capk)
            return fail(PSCL_EDEVICE, "retry chain %d: %lld entries exceed its state (%lld)", k, (long long)nk,
                        (long long)capk);
        HIP_TRY(hipStreamWaitEvent(h->retry_stream[cs + k], h->ev_base[p], 0));
        DlState T = b.S[cs + k];
        T.act = b.act[p] + (k ? A0 : 0);
        int r2 = dl_retry_chunk(h, T, k ? A - A0 : A0, a.rounds, a.d_llr, a.d_best, a.d_flags, a.d_attempts,
                                a.d_tried, a.tried_stride, d_cdl, h->retry_stream[cs + k],
                                (h->tune[PSCL_TUNE_DL_STREAMS] & 1) ? h->retry_stream[cs + k] : h->side_stream[cs + k],
                                h->ev_scr[cs + k], h->ev_def[cs + k], a.pipe, beside);
        if (r2) return r2;
    }
    if (parts == 2) {  // both chains done before the parity's indices are reused
        HIP_TRY(hipEventRecord(h->ev_join[cs >> 1], h->retry_stream[cs + 1]));
        HIP_TRY(hipStreamWaitEvent(h->retry_stream[cs], h->ev_join[cs >> 1], 0));
    }
    HIP_TRY(hipEventRecord(h->ev_retry[p], h->retry_stream[cs]));
    return PSCL_OK;
}

// a pipelined call's retry chains and DL counters, enqueued on the retry streams (ev_dl marks
// their end; join_pipe orders it into the handle's stream); beside: the next call's baseline is on
// the handle's stream, concurrent with them
int dl_enqueue_deferred(pscl_handle* h, bool beside) {
    if (!h->dl_defer_valid) return PSCL_OK;
    h->dl_defer_valid = false;
    const pscl_dl_call a = h->dl_defer;
    DlBufs b;
    int rc = dl_setup(h, a, b);  // (the sizes of the call's own setup: no allocation)
    if (rc) return rc;
    if ((rc = dl_chain(h, a, b, 0, beside))) return rc;
    hipStream_t rs = h->retry_stream[2 * dl_set(h, a, 0)];
    if (a.d_ref) {
        hipError_t e = pscl_launch_dl_count(a.d_best, a.d_flags, a.d_ref, a.B, h->W, a.k_payload, a.d_counters_dl, rs);
        if (e != hipSuccess) return fail(PSCL_EDEVICE, "dl_count launch: %s", hipGetErrorString(e));
    }
    HIP_TRY(hipEventRecord(h->ev_dl[a.pbase], rs));
    h->dl_pending[a.pbase] = true;
    return PSCL_OK;
}
}  // namespace

namespace {
// the fused TX of a pscl_simulate_device block (PSCL_TUNE_TX_FUSED): the baseline decode draws the
// rows it decodes (scl128_lane.hip TXF), writes the message words to d_ref's buffer and the rows of
// failing and deferred frames to d_llr's, and counts the uncoded baseline into unc
struct TxSpec {
    uint32_t k0 = 0, k1 = 0;
    int64_t frame0 = 0;
    double sigma = 0.0, scale = 0.0, unc_sigma = 0.0;
    int kp = 0;
    double* rows = nullptr;
    uint64_t* msg = nullptr;
    int64_t* unc = nullptr;  // [PSCL_NCOUNT] or null
};
int dlscl_impl(pscl_handle* h, const double* d_llr, int64_t B, int retries, uint64_t* d_best, uint8_t* d_flags,
               int32_t* d_attempts, int32_t* d_tried, int tried_stride, const uint64_t* d_ref, int k_payload,
               int64_t* d_counters_scl, int64_t* d_counters_dl, const TxSpec* tx);
}  // namespace

#ifndef PSCL_DL_TAIL_STREAM
#define PSCL_DL_TAIL_STREAM 1
#endif

int pscl_dlscl_device(pscl_handle* h, const double* d_llr, int64_t B, int retries, uint64_t* d_best, uint8_t* d_flags,
                      int32_t* d_attempts, int32_t* d_tried, int tried_stride, const uint64_t* d_ref, int k_payload,
                      int64_t* d_counters_scl, int64_t* d_counters_dl) {
    return dlscl_impl(h, d_llr, B, retries, d_best, d_flags, d_attempts, d_tried, tried_stride, d_ref, k_payload,
                      d_counters_scl, d_counters_dl, nullptr);
}

namespace {
int dlscl_impl(pscl_handle* h, const double* d_llr, int64_t B, int retries, uint64_t* d_best, uint8_t* d_flags,
               int32_t* d_attempts, int32_t* d_tried, int tried_stride, const uint64_t* d_ref, int k_payload,
               int64_t* d_counters_scl, int64_t* d_counters_dl, const TxSpec* tx) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    if (B < 0) return fail(PSCL_EINVAL, "B must be >= 0");
    if (B == 0) return PSCL_OK;
    if (!d_llr || !d_best || !d_flags) return fail(PSCL_EINVAL, "d_llr, d_best and d_flags are required");
    if (d_ref && (!d_counters_scl || !d_counters_dl)) return fail(PSCL_EINVAL, "d_ref given without both counters");
    if (k_payload < 0 || k_payload > h->K) return fail(PSCL_EINVAL, "k_payload out of range");
    const int rounds = h->crc_poly && retries > 0 ? (retries < h->K ? retries : h->K) : 0;
    if (d_tried && tried_stride < rounds) return fail(PSCL_EINVAL, "tried_stride < min(retries, K)");
    if (B > INT32_MAX) return fail(PSCL_EUNSUP, "B exceeds 2^31-1");
    struct HostClock {  // pscl_host_stats: this call's wall time on the host
        pscl_handle* h;
        std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
        ~HostClock() {
            h->host_call_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            h->host_calls++;
        }
    } host_clock{h};
    int rc = set_device(h);
    if (rc) return rc;
    pscl_dl_call a;
    a.d_llr = d_llr;
    a.B = B;
    a.rounds = rounds;
    a.d_best = d_best;
    a.d_flags = d_flags;
    a.d_attempts = d_attempts;
    a.d_tried = d_tried;
    a.tried_stride = tried_stride;
    a.d_ref = d_ref;
    a.k_payload = k_payload;
    a.d_counters_dl = d_counters_dl;
    // Chunks (tuning knob PSCL_TUNE_DL_CHUNKS, default 1): the baseline decodes run in order on the handle's
    // stream; the retry entries of chunk c are split over two chains, each on its own retry
    // stream with its own state, so the two chains' rounds overlap each other (and chunk c + 1's
    // baseline decode).  A round is latency-bound (a few 10^4 entries per launch), so a second
    // concurrent chain fills what one leaves idle.  PSCL_TUNE_DL_SPLIT (1 or 2) sets the chains per
    // chunk; chunks below 2 * kMinSplit failing frames keep one chain.  The default is 2 for a
    // blocking call and 1 when pipelined: there the previous call's chains already overlap this
    // one's, and a second chain per call only doubles the host's launches (config 4 measured
    // 2.65 -> 2.38 ms/step with one).
    a.nch = 1;
    a.nsplit = h->N > PSCL_FAST_N ? 0 : (h->pipelined ? 1 : 2);
    if (rounds > 0 && h->tune[PSCL_TUNE_DL_CHUNKS]) a.nch = h->tune[PSCL_TUNE_DL_CHUNKS];
    if (rounds > 0 && h->N <= PSCL_FAST_N && h->tune[PSCL_TUNE_DL_SPLIT]) a.nsplit = (int)h->tune[PSCL_TUNE_DL_SPLIT];
    a.cap = (B + a.nch - 1) / a.nch;
    // Pipelined (pscl_set_pipelined, one chunk): the call enqueues its baseline, then the retry
    // chains of the PREVIOUS pipelined call (whose baseline has ended or is about to: the host
    // waits only for that one), and leaves its own chains to the next call or join -- so the
    // handle's stream holds back-to-back baselines and the chains (high-priority streams) run
    // beside them, the host never waiting for the baseline it has just enqueued.
    a.pipe = h->pipelined && rounds > 0 && a.nch == 1;
    if (h->dl_defer_valid &&
        (!a.pipe || h->dl_defer.B != B || h->dl_defer.rounds != rounds || h->dl_defer.nsplit != a.nsplit)) {
        // (a different shape: the pending chains first, their state sized as they were)
        if ((rc = dl_enqueue_deferred(h))) return rc;
    }
    if ((rc = join_pipe(h, a.pipe ? 1 : 3))) return rc;
    a.pbase = a.pipe ? h->dl_par : 0;  // compaction parity of chunk 0
    if (a.pipe) {
        // the chains of the call dl_back calls back may still write their call's outputs (and, kDlPar
        // back, read this parity's compaction output): they end before this call starts (the
        // contract of pscl_set_pipelined: a call's buffers are free again at the dl_back-th following
        // call).  Consecutive calls' chains run concurrently (two chain sets, dl_set), so one call's
        // end does not cover another's; the invariant is by induction instead: every call makes the
        // handle's stream wait for the chains dl_back calls back (ev_dl, here), so any call further
        // back was already waited for by an earlier call; and calls whose pbase has the same parity
        // share one set's streams and DlState, which stream order keeps apart.
        // (PSCL_TUNE_DL_STREAMS bit 2 collapses everything to one set: chains then run in call order.)
        const int q = (a.pbase + kDlPar - h->dl_back) % kDlPar;
        if (h->dl_pending[q]) {
            HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_dl[q], 0));
            h->dl_pending[q] = false;
        }
        if (h->dl_pending[a.pbase]) {
            HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_dl[a.pbase], 0));
            h->dl_pending[a.pbase] = false;
        }
    }
    const int W = h->W;
    const int64_t row = h->rm_E ? h->rm_E : h->N;
    const int64_t nch = a.nch, cap = a.cap;
    hipStream_t s = h->stream;
    hipError_t e;
    if (d_attempts) HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)d_attempts, 1, (size_t)B, s));
    if (d_tried) HIP_TRY(hipMemsetAsync(d_tried, 0xff, (size_t)B * tried_stride * 4, s));
    DlBufs bufs;
    if (rounds > 0 && (rc = dl_setup(h, a, bufs))) return rc;
    for (int64_t c = 0; c < nch; ++c) {
        const int64_t c0 = c * cap, nc = (B - c0) < cap ? (B - c0) : cap;
        // baseline SCL (flip.py:79-80) of chunk c
        pscl_decode_params P;
        fill_decode_params(h, P, 0);
        P.llr = d_llr + c0 * row;
        P.B = nc;
        P.best = d_best + c0 * W;
        P.flags = d_flags + c0;
        P.ref = d_ref ? d_ref + c0 * W : nullptr;
        P.k_payload = k_payload;
        P.counters = d_counters_scl;
        // (N = 128: the DL-SCL baseline's screening kernel, PSCL_TUNE_DL_LANE; by default the
        // lane-per-path one at L = 8 and the two-lanes-per-path one at L = 4, which measured faster
        // beside the retry chains)
        if (rounds > 0) {
            const int64_t dl_lane = h->tune[PSCL_TUNE_DL_LANE] ? h->tune[PSCL_TUNE_DL_LANE]
                                                               : (PSCL_DL_LANE_DEFAULT ? PSCL_DL_LANE_DEFAULT : (h->L == 8 ? 1 : 2));
            P.no_lane = dl_lane != 1;
        }
        if (tx) {  // the fused TX: the lane kernel draws the chunk's rows (simulate_enqueue checked it applies)
            P.no_lane = 0;
            P.tx = 1;
            P.tx_k0 = tx->k0;
            P.tx_k1 = tx->k1;
            P.tx_kp = tx->kp;
            P.tx_crc_deg = h->crc_deg;
            P.tx_frame0 = tx->frame0 + c0;
            P.tx_sigma = tx->sigma;
            P.tx_scale = tx->scale;
            P.tx_unc_sigma = tx->unc_sigma;
            P.tx_crctab = h->d_crctab;
            P.tx_xtab = h->d_xtab;
            P.tx_rows = tx->rows + c0 * row;
            P.tx_msg = tx->msg + c0 * W;
            P.tx_unc_counters = tx->unc;
        }
        if (pscl_decode_wpg(P) < 1) return fail(PSCL_EUNSUP, "LDS budget exceeded (L=%d, K=%d)", h->L, h->K);
        // a pipelined call's baseline tail (re-decode, compaction, count) on tail_stream: the next
        // call's baseline follows this one's screening pass directly
        hipStream_t ts = s;
        const int tpar = a.pbase & 1;
        if (a.pipe && PSCL_DL_TAIL_STREAM && !h->tune[PSCL_TUNE_DL_TAIL]) {
            if (!h->tail_stream) {
                HIP_TRY(create_priority_stream(h, &h->tail_stream));
                for (int i = 0; i < 2; ++i) {
                    HIP_TRY(hipEventCreateWithFlags(&h->ev_tscr[i], hipEventDisableTiming));
                    HIP_TRY(hipEventCreateWithFlags(&h->ev_tail[i], hipEventDisableTiming));
                }
            }
            ts = h->tail_stream;
        }
        if ((rc = launch_decode(h, P, 0, s, 38, false, ts != s ? ts : nullptr, tpar))) return rc;
        if (ts != s && rounds <= 0) {  // (no compaction: the tail ends with the re-decode)
            HIP_TRY(hipEventRecord(h->ev_tail[tpar], ts));
            h->tail_pending[tpar] = true;
        }
        if (rounds > 0) {
            const int p = dl_parity(a, c);
            if (c >= 2) HIP_TRY(hipStreamWaitEvent(ts, h->ev_retry[p], 0));  // the parity's indices free again
            HIP_TRY(hipMemsetAsync(bufs.cnt[p], 0, 4, ts));
            if ((e = pscl_launch_dl_compact(d_flags + c0, nc, c0, bufs.act[p], nullptr, bufs.cnt[p], ts)) != hipSuccess)
                return fail(PSCL_EDEVICE, "dl_compact launch: %s", hipGetErrorString(e));
            // fused TX: the failing frames' rows, read by the retry chain (entries hold call-level frame
            // indices c0 + f)
            if (tx && (e = pscl_launch_tx_rows(P, bufs.act[p], bufs.cnt[p], nc, tx->rows, tx->frame0, ts)) != hipSuccess)
                return fail(PSCL_EDEVICE, "tx_rows launch: %s", hipGetErrorString(e));
            HIP_TRY(hipMemcpyAsync(h->h_count + p, bufs.cnt[p], 4, hipMemcpyDeviceToHost, ts));
            HIP_TRY(hipEventRecord(h->ev_base[p], ts));
            if (ts != s) {
                HIP_TRY(hipEventRecord(h->ev_tail[tpar], ts));
                h->tail_pending[tpar] = true;
            }
            if (c >= 1 && (rc = dl_chain(h, a, bufs, c - 1, true))) return rc;
        }
    }
    if (a.pipe) {
        // the previous call's chains now (its baseline precedes this call's on the stream), this
        // call's at the next call or join
        if ((rc = dl_enqueue_deferred(h, true))) return rc;
        h->dl_defer = a;
        h->dl_defer_valid = true;
        h->dl_par = (h->dl_par + 1) % kDlPar;
        return PSCL_OK;
    }
    if (rounds > 0) {
        if ((rc = dl_chain(h, a, bufs, nch - 1, false))) return rc;
        // (the chunk chains alternate two sets: the last two end every chain)
        HIP_TRY(hipStreamWaitEvent(s, h->ev_retry[dl_parity(a, nch - 1)], 0));
        if (nch >= 2) HIP_TRY(hipStreamWaitEvent(s, h->ev_retry[dl_parity(a, nch - 2)], 0));
    }
    if (d_ref) {
        e = pscl_launch_dl_count(d_best, d_flags, d_ref, B, W, k_payload, d_counters_dl, s);
        if (e != hipSuccess) return fail(PSCL_EDEVICE, "dl_count launch: %s", hipGetErrorString(e));
    }
    return PSCL_OK;
}
}  // namespace

static int decode_host(pscl_handle* h, const double* llr, int64_t B, const int8_t* forced, int32_t* n_paths,
                       int8_t* best_bits, uint8_t* crc_pass, int32_t* best_idx, double* metrics, int8_t* cands,
                       double* info_llrs, int sc_hard) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    if (B < 0) return fail(PSCL_EINVAL, "B must be >= 0");
    if (B == 0) return PSCL_OK;
    if (!llr || !n_paths) return fail(PSCL_EINVAL, "llr and n_paths are required");
    const int K = h->K, L = h->L, W = h->W, N = h->N;
    std::vector<uint64_t> hforce;
    if (forced) {
        hforce.assign((size_t)B * 2 * W, 0);
        for (int64_t b = 0; b < B; ++b) {
            uint64_t* fr = &hforce[(size_t)b * 2 * W];
            for (int jj = 0; jj < K; ++jj) {
                int v = forced[b * K + jj];
                if (v == 0 || v == 1) {
                    fr[jj >> 6] |= 1ULL << (jj & 63);
                    if (v) fr[W + (jj >> 6)] |= 1ULL << (jj & 63);
                } else if (v != -1) {
                    return fail(PSCL_EINVAL, "force_info_bits entries must be -1, 0, or 1");
                }
            }
        }
    }
    int rc = enter(h);
    if (rc) return rc;
    void *d_llr, *d_force = nullptr, *d_np, *d_best, *d_flags, *d_met = nullptr, *d_cands = nullptr, *d_illr = nullptr;
    const size_t sz_llr = (size_t)B * (h->rm_E ? h->rm_E : N) * 8;
    if ((rc = ensure(h, 0, sz_llr, &d_llr))) return rc;
    if (forced && (rc = ensure(h, 1, hforce.size() * 8, &d_force))) return rc;
    if ((rc = ensure(h, 2, (size_t)B * 4, &d_np))) return rc;
    if ((rc = ensure(h, 3, (size_t)B * W * 8, &d_best))) return rc;
    if ((rc = ensure(h, 4, (size_t)B, &d_flags))) return rc;
    if (metrics && (rc = ensure(h, 5, (size_t)B * L * 8, &d_met))) return rc;
    if (cands && (rc = ensure(h, 6, (size_t)B * L * W * 8, &d_cands))) return rc;
    if (info_llrs && (rc = ensure(h, 7, (size_t)B * L * (K > 0 ? K : 1) * 8, &d_illr))) return rc;
    HIP_TRY(hipMemcpyAsync(d_llr, llr, sz_llr, hipMemcpyHostToDevice, h->stream));
    if (forced) HIP_TRY(hipMemcpyAsync(d_force, hforce.data(), hforce.size() * 8, hipMemcpyHostToDevice, h->stream));
    const int hist = info_llrs != nullptr;
    pscl_decode_params P;
    fill_decode_params(h, P, hist);
    P.llr = (const double*)d_llr;
    P.B = B;
    P.force = (const uint64_t*)d_force;
    P.n_paths = (int32_t*)d_np;
    P.best = (uint64_t*)d_best;
    P.flags = (uint8_t*)d_flags;
    P.metrics = (double*)d_met;
    P.cands = (uint64_t*)d_cands;
    P.info_llrs = (double*)d_illr;
    P.sc_hard = sc_hard;
    if (pscl_decode_wpg(P) < 1) return fail(PSCL_EUNSUP, "LDS budget exceeded (L=%d, K=%d)", h->L, h->K);
    if ((rc = launch_decode(h, P, hist))) return rc;
    std::vector<int32_t> hnp((size_t)B);
    std::vector<uint64_t> hbest((size_t)B * W);
    std::vector<uint8_t> hflags((size_t)B);
    HIP_TRY(hipMemcpyAsync(hnp.data(), d_np, (size_t)B * 4, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipMemcpyAsync(hbest.data(), d_best, (size_t)B * W * 8, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipMemcpyAsync(hflags.data(), d_flags, (size_t)B, hipMemcpyDeviceToHost, h->stream));
    std::vector<uint64_t> hc;
    if (cands) {
        hc.resize((size_t)B * L * W);
        HIP_TRY(hipMemcpyAsync(hc.data(), d_cands, hc.size() * 8, hipMemcpyDeviceToHost, h->stream));
    }
    if (metrics) HIP_TRY(hipMemcpyAsync(metrics, d_met, (size_t)B * L * 8, hipMemcpyDeviceToHost, h->stream));
    if (info_llrs)
        HIP_TRY(hipMemcpyAsync(info_llrs, d_illr, (size_t)B * L * K * 8, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    for (int64_t b = 0; b < B; ++b) {
        n_paths[b] = hnp[(size_t)b];
        if (best_bits)
            for (int jj = 0; jj < K; ++jj)
                best_bits[b * K + jj] = (int8_t)((hbest[(size_t)b * W + (jj >> 6)] >> (jj & 63)) & 1);
        if (crc_pass) crc_pass[b] = (hflags[(size_t)b] & PSCL_FLAG_CRC_PASS) ? 1 : 0;
        if (best_idx) best_idx[b] = (int32_t)(hflags[(size_t)b] & PSCL_FLAG_IDX_MASK);
        if (cands)
            for (int r = 0; r < L; ++r)
                for (int jj = 0; jj < K; ++jj)
                    cands[((size_t)b * L + r) * K + jj] =
                        (int8_t)((hc[((size_t)b * L + r) * W + (jj >> 6)] >> (jj & 63)) & 1);
    }
    return PSCL_OK;
}

int pscl_decode(pscl_handle* h, const double* llr, int64_t B, const int8_t* forced, int32_t* n_paths,
                int8_t* best_bits, uint8_t* crc_pass, int32_t* best_idx, double* metrics, int8_t* cands,
                double* info_llrs) {
    return decode_host(h, llr, B, forced, n_paths, best_bits, crc_pass, best_idx, metrics, cands, info_llrs, 0);
}

int pscl_sc_decode(pscl_handle* h, const double* llr, int64_t B, int8_t* bits) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    if (B <= 0) return B < 0 ? fail(PSCL_EINVAL, "B must be >= 0") : PSCL_OK;
    std::vector<int32_t> np((size_t)B);
    return decode_host(h, llr, B, nullptr, np.data(), bits, nullptr, nullptr, nullptr, nullptr, nullptr, 1);
}

namespace {
int uncoded_launch(pscl_handle* h, uint64_t seed, uint32_t stream_id, double ebno_db, int k_payload, int64_t frame0,
                   int64_t B, int64_t* d_counters, bool no_enter);
}

int pscl_uncoded_device(pscl_handle* h, uint64_t seed, uint32_t stream_id, double ebno_db, int k_payload,
                        int64_t frame0, int64_t B, int64_t* d_counters) {
    return uncoded_launch(h, seed, stream_id, ebno_db, k_payload, frame0, B, d_counters, false);
}

namespace {
int uncoded_launch(pscl_handle* h, uint64_t seed, uint32_t stream_id, double ebno_db, int k_payload, int64_t frame0,
                   int64_t B, int64_t* d_counters, bool no_enter) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    if (B < 0 || frame0 < 0) return fail(PSCL_EINVAL, "B and frame0 must be >= 0");
    if (B == 0) return PSCL_OK;
    if (!d_counters) return fail(PSCL_EINVAL, "d_counters is NULL");
    if (k_payload < 0 || k_payload > PSCL_MAX_N) return fail(PSCL_EINVAL, "k_payload out of range");
    int rc = no_enter ? set_device(h) : enter(h);
    if (rc) return rc;
    pscl_channel_params P;
    memset(&P, 0, sizeof(P));
    P.seed = seed;
    P.stream_id = stream_id;
    P.k_payload = k_payload;
    const double ebno = pow(10.0, ebno_db / 10.0);
    P.noise_var = 1.0 / (2.0 * ebno);  // run_fer_sweep.py:66-67
    P.sigma = sqrt(P.noise_var);
    P.frame0 = frame0;
    P.B = B;
    hipError_t e = pscl_launch_uncoded(P, d_counters, h->stream);
    if (e != hipSuccess) return fail(PSCL_EDEVICE, "uncoded kernel launch: %s", hipGetErrorString(e));
    return PSCL_OK;
}
}  // namespace

namespace {
int channel_launch(pscl_handle* h, uint64_t seed, uint32_t stream_id, double ebno_db, double rate, int k_payload,
                   int64_t frame0, int64_t B, double* d_llr, uint64_t* d_msg, int64_t* d_unc, bool no_enter = false);

#ifndef PSCL_TX_FUSED_DEFAULT
#define PSCL_TX_FUSED_DEFAULT 0
#endif
// whether a pscl_simulate[_device] block takes the fused TX (PSCL_TUNE_TX_FUSED, default
// PSCL_TX_FUSED_DEFAULT): its baseline decode must be the screening lane kernel of the (128,64) code
// on plain rows (L = 4 or 8), which then draws the rows itself
bool tx_fused_applies(const pscl_handle* h, int k_payload) {
    const int64_t k = h->tune[PSCL_TUNE_TX_FUSED];
    if (!(k == 1 || (k == 0 && PSCL_TX_FUSED_DEFAULT))) return false;
    if (h->N != 128 || h->rm_E || !h->screen || (h->L != 8 && h->L != 4) || k_payload + h->crc_deg != h->K) return false;
    pscl_decode_params T;
    fill_decode_params(h, T, 0);
    T.B = 1;
    T.apx = 1;
    return pscl_lane_available(T) != 0;
}

// One SNR point of run_sweep enqueued (pscl_simulate / pscl_simulate_device): chunks of at most
// 2^20 frames through handle scratch (N * 8 bytes of LLRs per frame: about 1 GiB per chunk at
// N = 128), each = TX (+ the uncoded baseline) + pscl_dlscl_device.  On a pipelined handle every
// chunk is one pipelined DL-SCL call: its retry chains overlap the next chunk's (or the next
// point's) TX and baseline, so kDlPar scratch sets rotate with the DL-SCL call parity, and a set
// is rewritten only after the chains of the call kDlPar back that used it have ended.
int simulate_enqueue(pscl_handle* h, uint64_t seed, uint32_t stream_id, double ebno_db, double rate, int k_payload,
                     int64_t frame0, int64_t B, int retries, int include_uncoded, int64_t* cs) {
    const int64_t chunk = B < (1 << 20) ? B : (1 << 20);
    const int W = h->W, N = h->N;
    int rc;
    for (int64_t f = 0; f < B; f += chunk) {
        const int64_t n = B - f < chunk ? B - f : chunk;
        const int par = h->pipelined ? h->dl_par : 0;
        if (h->pipelined && h->dl_pending[par]) {  // (the chains that last read this scratch set)
            HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_dl[par], 0));
            h->dl_pending[par] = false;
        }
        static const int kSimSlot[kDlPar] = {30, 66, 84, 88};
        void *d_llr, *d_msg, *d_best, *d_flags;
        // (pipelined: every parity's set sized at once, so the first call warms all of them and no
        // later call of a sweep allocates -- ~130 us of hipMalloc on the host per new set)
        for (int q = h->pipelined ? 0 : par; q <= (h->pipelined ? kDlPar - 1 : par); ++q) {
            const int base = kSimSlot[q];
            if ((rc = ensure(h, base, (size_t)chunk * N * 8, &d_llr))) return rc;
            if ((rc = ensure(h, base + 1, (size_t)chunk * W * 8, &d_msg))) return rc;
            if ((rc = ensure(h, base + 2, (size_t)chunk * W * 8, &d_best))) return rc;
            if ((rc = ensure(h, base + 3, (size_t)chunk, &d_flags))) return rc;
        }
        const int base = kSimSlot[par];
        if ((rc = ensure(h, base, (size_t)chunk * N * 8, &d_llr))) return rc;
        if ((rc = ensure(h, base + 1, (size_t)chunk * W * 8, &d_msg))) return rc;
        if ((rc = ensure(h, base + 2, (size_t)chunk * W * 8, &d_best))) return rc;
        if ((rc = ensure(h, base + 3, (size_t)chunk, &d_flags))) return rc;
        // the fused TX (PSCL_TUNE_TX_FUSED): the baseline decode draws the rows itself -- where its
        // screening launch is the lane kernel of the (128,64) code on plain rows
        TxSpec tx;
        const bool fused = tx_fused_applies(h, k_payload);
        if (fused) {
            h->n_fused_tx++;
            tx.k0 = (uint32_t)seed;
            tx.k1 = (uint32_t)(seed >> 32) ^ (stream_id * 0x85EBCA6Bu);  // (channel_kernel's key)
            tx.frame0 = frame0 + f;
            const double ebno = pow(10.0, ebno_db / 10.0);
            const double nv = 1.0 / (2.0 * rate * ebno);  // (channel_launch's parameters)
            tx.sigma = sqrt(nv);
            tx.scale = 2.0 / nv;
            tx.unc_sigma = sqrt(1.0 / (2.0 * ebno));
            tx.kp = k_payload;
            tx.rows = (double*)d_llr;
            tx.msg = (uint64_t*)d_msg;
            tx.unc = include_uncoded ? cs + 2 * PSCL_NCOUNT : nullptr;
        } else {
            // N <= 128: the uncoded baseline is counted by the TX launch itself (same payload draw)
            const bool unc_fused = include_uncoded && N <= PSCL_FAST_N;
            if ((rc = channel_launch(h, seed, stream_id, ebno_db, rate, k_payload, frame0 + f, n, (double*)d_llr,
                                     (uint64_t*)d_msg, unc_fused ? cs + 2 * PSCL_NCOUNT : nullptr, true)))
                return rc;
            if (include_uncoded && !unc_fused &&
                (rc = uncoded_launch(h, seed, stream_id, ebno_db, k_payload, frame0 + f, n, cs + 2 * PSCL_NCOUNT, true)))
                return rc;
        }
        const int back = h->dl_back;
        h->dl_back = kDlPar;  // (its own scratch set: kDlPar sets rotate with the call parity)
        rc = dlscl_impl(h, (const double*)d_llr, n, retries, (uint64_t*)d_best, (uint8_t*)d_flags, nullptr, nullptr, 0,
                        (const uint64_t*)d_msg, k_payload, cs, cs + PSCL_NCOUNT, fused ? &tx : nullptr);
        h->dl_back = back;
        if (rc) return rc;
    }
    return PSCL_OK;
}
}  // namespace

int pscl_simulate_device(pscl_handle* h, uint64_t seed, uint32_t stream_id, double ebno_db, double rate, int k_payload,
                         int64_t frame0, int64_t B, int retries, int include_uncoded, int64_t* d_counters) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    if (!d_counters) return fail(PSCL_EINVAL, "d_counters is NULL");
    if (B < 0 || frame0 < 0) return fail(PSCL_EINVAL, "B and frame0 must be >= 0");
    if (B == 0) return PSCL_OK;
    int rc = set_device(h);
    if (rc) return rc;
    if ((rc = join_pipe(h, 1))) return rc;  // (plain decodes' pending re-decodes; DL chains keep overlapping)
    return simulate_enqueue(h, seed, stream_id, ebno_db, rate, k_payload, frame0, B, retries, include_uncoded, d_counters);
}

int pscl_simulate(pscl_handle* h, uint64_t seed, uint32_t stream_id, double ebno_db, double rate, int k_payload,
                  int64_t frame0, int64_t B, int retries, int include_uncoded, int64_t* counters) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    if (!counters) return fail(PSCL_EINVAL, "counters is NULL");
    if (B < 0 || frame0 < 0) return fail(PSCL_EINVAL, "B and frame0 must be >= 0");
    memset(counters, 0, sizeof(int64_t) * 3 * PSCL_NCOUNT);
    if (B == 0) return PSCL_OK;
    int rc = enter(h);
    if (rc) return rc;
    void* d_cnt;
    if ((rc = ensure(h, 34, sizeof(int64_t) * 3 * PSCL_NCOUNT, &d_cnt))) return rc;
    HIP_TRY(hipMemsetAsync(d_cnt, 0, sizeof(int64_t) * 3 * PSCL_NCOUNT, h->stream));
    if ((rc = simulate_enqueue(h, seed, stream_id, ebno_db, rate, k_payload, frame0, B, retries, include_uncoded,
                               (int64_t*)d_cnt)))
        return rc;
    if ((rc = join_pipe(h))) return rc;  // (a pipelined handle: this call's chains, then the counters)
    HIP_TRY(hipMemcpyAsync(counters, d_cnt, sizeof(int64_t) * 3 * PSCL_NCOUNT, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    return PSCL_OK;
}

namespace {
// the TX launch (pscl_channel_device); d_unc != null also counts the uncoded baseline of the
// same frames (N <= 128: channel_kernel's phase A); no_enter: pending pipelined DL-SCL chains stay
// where they are (pscl_simulate_device: they overlap this TX)
int channel_launch(pscl_handle* h, uint64_t seed, uint32_t stream_id, double ebno_db, double rate, int k_payload,
                   int64_t frame0, int64_t B, double* d_llr, uint64_t* d_msg, int64_t* d_unc, bool no_enter) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    if (B < 0 || frame0 < 0) return fail(PSCL_EINVAL, "B and frame0 must be >= 0");
    if (B == 0) return PSCL_OK;
    if (!d_llr) return fail(PSCL_EINVAL, "d_llr is NULL");
    if (!(rate > 0)) return fail(PSCL_EINVAL, "rate must be positive");
    if (k_payload + h->crc_deg != h->K || k_payload < 0)
        return fail(PSCL_EINVAL, "k_payload (%d) + crc degree (%d) must equal K (%d)", k_payload, h->crc_deg, h->K);
    int rc = no_enter ? set_device(h) : enter(h);
    if (rc) return rc;
    pscl_channel_params P;
    memset(&P, 0, sizeof(P));
    P.seed = seed;
    P.stream_id = stream_id;
    P.N = h->N;
    P.K = h->K;
    P.W = h->W;
    P.k_payload = k_payload;
    P.crc_deg = h->crc_deg;
    P.xtab = h->d_xtab;
    P.crctab = h->d_crctab;
    const double ebno = pow(10.0, ebno_db / 10.0);
    P.noise_var = 1.0 / (2.0 * rate * ebno);
    P.sigma = sqrt(P.noise_var);
    P.llr_scale = 2.0 / P.noise_var;
    P.frame0 = frame0;
    P.B = B;
    P.llr = d_llr;
    P.msg = d_msg;
    P.rm_E = h->rm_E;
    P.rm_order = h->d_rm_order;
    if (d_unc) {
        P.unc_counters = d_unc;
        P.unc_sigma = sqrt(1.0 / (2.0 * ebno));  // run_fer_sweep.py:66-67 (uncoded: R = 1)
    }
    hipError_t e = pscl_launch_channel(P, h->stream);
    if (e != hipSuccess) return fail(PSCL_EDEVICE, "channel kernel launch: %s", hipGetErrorString(e));
    return PSCL_OK;
}
}  // namespace

int pscl_channel_device(pscl_handle* h, uint64_t seed, uint32_t stream_id, double ebno_db, double rate, int k_payload,
                        int64_t frame0, int64_t B, double* d_llr, uint64_t* d_msg) {
    return channel_launch(h, seed, stream_id, ebno_db, rate, k_payload, frame0, B, d_llr, d_msg, nullptr);
}

int pscl_set_rate_match(pscl_handle* h, int E) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    if (E < 0) return fail(PSCL_EINVAL, "E must be >= 0");
    if (E > 0 && E > h->N && h->N < 32)
        return fail(PSCL_EUNSUP, "repetition (E > N) needs N >= 32 (sub-block interleaver without padding)");
    if (E == h->rm_E) return PSCL_OK;
    // (the interleaver tables depend on N only: uploaded by pscl_create; enqueued launches carry
    // rm_E in their parameter block.  A pipelined DL-SCL call's retry chains are not enqueued yet --
    // they are built from the handle at the next call or join -- so they are enqueued here first,
    // with the rate matching their call's LLR rows were written for)
    const int rc = enter(h);
    if (rc) return rc;
    h->rm_E = E;
    return PSCL_OK;
}

int pscl_device_alloc(pscl_handle* h, void** d_ptr, int64_t bytes) {
    if (!h || !d_ptr || bytes < 0) return fail(PSCL_EINVAL, "bad arguments");
    int rc = enter(h);
    if (rc) return rc;
    HIP_TRY(hipMalloc(d_ptr, (size_t)(bytes > 0 ? bytes : 1)));
    return PSCL_OK;
}

int pscl_device_free(pscl_handle* h, void* d_ptr) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    // pending pipelined work may still read or write the buffer (a deferred DL-SCL call's chains
    // hold its LLR, output, reference and counter pointers): enqueue it, then drain every stream
    int rc = enter(h);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(h->stream));
    quiesce(h);
    if (d_ptr) HIP_TRY(hipFree(d_ptr));
    return PSCL_OK;
}

int pscl_memcpy_htod(pscl_handle* h, void* d_dst, const void* src, int64_t bytes) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    int rc = enter(h);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(d_dst, src, (size_t)bytes, hipMemcpyHostToDevice, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    return PSCL_OK;
}

int pscl_memcpy_dtoh(pscl_handle* h, void* dst, const void* d_src, int64_t bytes) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    int rc = enter(h);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(dst, d_src, (size_t)bytes, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    return PSCL_OK;
}

int pscl_memset_device(pscl_handle* h, void* d_dst, int value, int64_t bytes) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    int rc = enter(h);
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync(d_dst, value, (size_t)bytes, h->stream));
    return PSCL_OK;
}

int pscl_set_screening(pscl_handle* h, int enable) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    h->screen = enable != 0;
    return PSCL_OK;
}

int pscl_screening_count(pscl_handle* h, int64_t* count) {
    if (!h || !count) return fail(PSCL_EINVAL, "bad arguments");
    *count = 0;
    if (!h->screened || !h->scratch[h->screened_slot].p) return PSCL_OK;
    int rc = enter(h);
    if (rc) return rc;
    int32_t c = 0;
    HIP_TRY(hipMemcpyAsync(&c, h->scratch[h->screened_slot].p, 4, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    *count = c;
    return PSCL_OK;
}

int pscl_softplus_tails_device(pscl_handle* h, const double* d_v, int64_t n, double* d_exact, double* d_apx) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    if (n < 0) return fail(PSCL_EINVAL, "n must be >= 0");
    if (n == 0) return PSCL_OK;
    if (!d_v || !d_exact || !d_apx) return fail(PSCL_EINVAL, "d_v, d_exact and d_apx are required");
    int rc = enter(h);
    if (rc) return rc;
    hipError_t e = pscl_launch_softplus_tails(d_v, n, h->d_exp_table, d_exact, d_apx, h->stream);
    if (e != hipSuccess) return fail(PSCL_EDEVICE, "softplus tails launch: %s", hipGetErrorString(e));
    return PSCL_OK;
}

namespace {
int tail_scan(pscl_handle* h, uint32_t lo, uint32_t hi, uint64_t* d_out, int bits) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    if (!d_out) return fail(PSCL_EINVAL, "d_out is required");
    if (lo > hi) return fail(PSCL_EINVAL, "lo > hi");
    int rc = enter(h);
    if (rc) return rc;
    hipError_t e =
        pscl_launch_tail_abs_scan(lo, hi, h->d_exp_table, reinterpret_cast<unsigned long long*>(d_out), h->stream, bits);
    if (e != hipSuccess) return fail(PSCL_EDEVICE, "tail scan launch: %s", hipGetErrorString(e));
    return PSCL_OK;
}
}  // namespace

int pscl_tail_abs_scan_device(pscl_handle* h, uint32_t lo, uint32_t hi, uint64_t* d_out) {
    return tail_scan(h, lo, hi, d_out, 0);
}

int pscl_tail2_scan_device(pscl_handle* h, uint32_t lo, uint32_t hi, uint64_t* d_out) {
    return tail_scan(h, lo, hi, d_out, 1);
}

int pscl_timing_enable(pscl_handle* h, int enable) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    h->timing = enable != 0;
    h->ev_used = 0;
    return PSCL_OK;
}

int pscl_timing_read_split(pscl_handle* h, int64_t* main_launches, double* main_ms, int64_t* side_launches,
                           double* side_ms) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    int rc = enter(h);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(h->stream));
    quiesce(h);
    double tot[2] = {0.0, 0.0};
    int64_t cnt[2] = {0, 0};
    for (size_t i = 0; i + 1 < h->ev_used; i += 2) {
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, h->ev_pool[i], h->ev_pool[i + 1]));
        const int m = h->ev_main[i / 2] ? 0 : 1;
        tot[m] += ms;
        ++cnt[m];
    }
    if (main_launches) *main_launches = cnt[0];
    if (main_ms) *main_ms = tot[0];
    if (side_launches) *side_launches = cnt[1];
    if (side_ms) *side_ms = tot[1];
    return PSCL_OK;
}

int pscl_timing_read(pscl_handle* h, int64_t* launches, double* total_ms) {
    if (!h || !launches || !total_ms) return fail(PSCL_EINVAL, "bad arguments");
    int64_t n0 = 0, n1 = 0;
    double t0 = 0.0, t1 = 0.0;
    const int rc = pscl_timing_read_split(h, &n0, &t0, &n1, &t1);
    if (rc) return rc;
    *launches = n0 + n1;
    *total_ms = t0 + t1;
    return PSCL_OK;
}

int pscl_host_stats(pscl_handle* h, double* call_ms, double* wait_ms, int64_t* calls, int reset) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    if (call_ms) *call_ms = h->host_call_ms;
    if (wait_ms) *wait_ms = h->host_wait_ms;
    if (calls) *calls = h->host_calls;
    if (reset) {
        h->host_call_ms = h->host_wait_ms = 0.0;
        h->host_calls = 0;
    }
    return PSCL_OK;
}

int pscl_path_stats(pscl_handle* h, int64_t* fused_post_rounds, int64_t* post_rounds, int64_t* fused_tx_blocks,
                    int64_t* post_epw4_launches, int64_t* lane_exact_launches) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    if (lane_exact_launches) *lane_exact_launches = h->n_lane_exact;
    if (post_epw4_launches) *post_epw4_launches = h->n_post_epw4;
    if (fused_post_rounds) *fused_post_rounds = h->n_fpost_rounds;
    if (post_rounds) *post_rounds = h->n_post_rounds;
    if (fused_tx_blocks) *fused_tx_blocks = h->n_fused_tx;
    return PSCL_OK;
}

int pscl_launch_info(pscl_handle* h, int64_t B, int* waves_per_wg, int64_t* grid, int* lds_bytes) {
    if (!h) return fail(PSCL_EINVAL, "NULL handle");
    pscl_decode_params P;
    fill_decode_params(h, P, 0);
    P.B = B;
    if (waves_per_wg) *waves_per_wg = pscl_decode_wpg(P);
    if (grid) *grid = pscl_decode_grid(P);
    if (lds_bytes) *lds_bytes = pscl_decode_lds(P, 0);
    return PSCL_OK;
}

}  // extern "C"
