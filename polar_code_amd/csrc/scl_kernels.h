// scl_kernels.h -- parameter blocks shared by the HIP kernels and the C-ABI layer.
#ifndef PSCL_SCL_KERNELS_H
#define PSCL_SCL_KERNELS_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "polar_scl.h"

#define PSCL_MAX_WAVES_PER_WG 4
// code length of the specialised, DL-SCL replay and TX kernels; longer codes decode in
// scl_long.hip
#define PSCL_FAST_N 128
// 1: the scl128 epilogue tables (u-byte gather, CRC syndrome) are staged in LDS per workgroup;
// 0: read from global memory
#ifndef PSCL_EPI_LDS
#define PSCL_EPI_LDS 1
#endif

// DL-SCL retry rounds (dlscl.hip, dl_post_kernel): entry e = one failing frame's retry state.
// One pass per round over the entries just decoded: replay of the attempt's best path (its
// leaf LLRs), final-attempt bookkeeping and the CRC stop rule, then for the survivors the next
// flip (q = |L0| @ beta), its force words, the warm-start state of its forced prefix and the
// append to the next round's bucket list.  init = 1: the first pass, over the baseline.
struct pscl_post_params {
    const double* llr;           // channel LLRs [.][N] (or [.][E] with rate matching)
    int N, n, K, W, rm_E;
    const int32_t* rm_src;
    uint64_t info_mask[2];
    const int32_t* info_set;     // [K] (device)
    const uint64_t* exp_table;   // glibc exp table (exact metric tails)
    int rounds;                  // min(retries, K)
    int narrow;                  // small workgroups, beta through L2 (pipelined calls, dl_post_kernel)
    int epw;                     // narrow form: entries per wavefront (2, 4; 0: PSCL_POST_EPW_NARROW)
    int warm_apx;                // 1: warm-start metrics from the screening tail (the main chain of a
                                 // screened chain, PSCL_TUNE_DL_WARM_APX), 0: exact
    int64_t grid_cap;            // 0, or the workgroup cap of a launch (tuning knob; default PSCL_POST_GRID)
    int64_t pairs;               // 0, or the entry pairs per wavefront the grid is sized for (tuning knob)
    int init;
    const int32_t* in_count;     // bucket counts of this round (init: unused, cap entries)
    const int32_t* in_list;      // bucket lists of this round ([NSEG][cap] entry ids)
    int64_t cap;
    int32_t* out_count;          // next round's bucket counts (zeroed)
    int32_t* out_list;           // [NSEG][cap]
    const int64_t* act;          // [cap] frame index (LLR row) of each entry
    uint64_t* tried;             // [cap][2] tried-index bit sets
    int32_t* ntried;             // [cap]
    const double* beta;          // [K][K] or null
    double beta_absmax;          // max |beta| (the flip metric certificate's bound)
    uint64_t* force;             // [cap][2][W]
    double* warm_metric;         // [cap][NSEG]
    uint64_t* warm_u;            // [cap][2]
    const uint64_t* ob;          // [cap][W] this round's best bits, by entry
    const uint8_t* of;           // [cap]
    uint64_t* best;              // [B][W] final best bits (per frame)
    uint8_t* flags;              // [B]
    int32_t* attempts;           // [B] or null
    int32_t* tried_out;          // [B][tried_stride] or null
    int tried_stride;
    int64_t* counters;           // or null: PSCL_CNT_RETRIES += decodes
};

struct pscl_decode_params {
    const double* llr;  // [B][N]
    int64_t B;
    int N, n, K, L, W;
    uint64_t info_mask[2];       // bit phi set <=> phase phi is an information bit
    const uint32_t* crc_cols;    // [K] check syndrome columns (zeros when no CRC)
    const int32_t* info_set;     // [K] information positions, ascending (device)
    int has_crc;
    int sc_hard;                 // 1: successive cancellation, hard decisions (L = 1 path)
    const uint64_t* exp_table;   // [256] glibc exp table (device)
    const uint64_t* force;       // [B][2][W] or null
    int32_t* n_paths;            // [B] or null
    uint64_t* best;              // [B][W] or null
    uint8_t* flags;              // [B] or null
    double* metrics;             // [B][L] or null
    uint64_t* cands;             // [B][L][W] or null
    double* info_llrs;           // [B][L][K] or null (needs the HIST kernel)
    double* best_info_llrs;      // [B][K] or null: the best path's decision LLRs (HIST kernel)
    const int64_t* fidx;         // [B] or null: frame b reads LLR row fidx[b] (outputs stay at b)
    const int32_t* d_count;      // or null: decode min(B, *d_count) frames (grid sized for B)
    int rm_E;                    // NR rate matching: received length E (0 = none; llr is [B][E])
    const int32_t* rm_src;       // [N] de-interleave source index k(i) into the de-rate-matched vector
    const uint64_t* ref;         // [B][W] or null
    int k_payload;
    int64_t* counters;           // [PSCL_NCOUNT] (device)
    const uint64_t* epi_table;   // scl128 epilogue tables (device): u-byte -> info-bit gather
                                 // [16][256] uint8, then ib-nibble -> CRC syndrome [K4][16] uint32
    int epi_words;               // 8-byte words of epi_table staged in LDS
    int wg_fixed_bytes;          // LDS per workgroup besides the wavefronts' (tables)
    int fast;                    // 1: the specialised N = 128, L <= 8 kernel (scl128.hip)
    int wave_bytes;              // LDS bytes per wavefront
    int a_bytes;                 // LDS bytes of the LLR slots per wavefront
    // screening decode (scl128 compiled-in codes, plain decodes): bounded-error metric tails,
    // frames whose list order is not certain are appended to amb_list instead of finishing
    int apx;
    int64_t* amb_list;           // [B] frame indices to re-decode exactly
    int32_t* amb_count;
    int32_t* amb_elist;          // or (bucket-list launches): [NSEG][bcap] entry ids by bucket, appended
                                 // instead (amb_count then [NSEG * CSTRIDE]); their flags PSCL_DL_DEFERRED
    int out_by_row;              // 1: outputs, reference words and counts at LLR row fidx[b]
    int wpg_cap;                 // 0, or an upper bound on the wavefronts per workgroup (tuning knob)
    int32_t* cpart;              // or (counting launches, P.ref): per-wavefront error counts [slots][4]
                                 // (frame, bit, payload-frame, payload-bit errors), stored instead of
                                 // added, summed by pscl_launch_count_reduce (no same-address atomics)
    int no_lane;                 // 1: a screening launch takes the two-lanes-per-path kernel even where
                                 // the lane-per-path one exists (PSCL_TUNE_DL_LANE)
    int64_t grid_cap;            // 0, or an upper bound on the workgroups of the launch (the
                                 // kernels stride over frames; a d_count launch of few frames)
    // code lengths above 128 (scl_long.hip): information set as N/64 words, and the global
    // scratch of one workgroup per frame in flight
    const uint64_t* info_words;  // [N/64] (device)
    unsigned char* long_scratch;  // [grid][long_block_bytes]
    int64_t long_block_bytes;
    int long_mode;               // 1: N > PSCL_FAST_N, scl_long.hip
    // DL-SCL retry rounds (dlscl.hip): the launch's frames are the entries of PSCL_DL_NSEG
    // bucket lists (bucket k at elist + k * bcap, bcount[k * PSCL_DL_CSTRIDE] entries), in
    // bucket order; frame i -> entry e, which indexes fidx (LLR row), force and the outputs.
    const int32_t* elist;
    const int32_t* bcount;
    int64_t bcap;
    // warm start (FS kernels with a compiled-in code): bucket k holds forced decodes whose
    // forced prefix covers phases [0, 16 k); a wavefront starts at phase 16 k of its first
    // frame's bucket with each frame's metric warm_metric[e][k] and bits warm_u[e][0..1]
    // below 16 k (the forced prefix's single path, replayed exactly by dl_post_kernel)
    const double* warm_metric;   // [entries][PSCL_DL_NSEG]
    const uint64_t* warm_u;      // [entries][2]
    // fused TX (pscl_simulate_device, PSCL_TUNE_TX_FUSED; the lane kernel of the (128,64) code): the
    // kernel draws frame b's channel row from channel_kernel's Philox stream (key tx_k0/tx_k1, frame
    // counter tx_frame0 + b) instead of loading it, bit for bit the row channel_kernel writes; it
    // writes the transmitted message of every frame to tx_msg (the launch's reference words: P.ref ==
    // tx_msg for the exact re-decode), the rows of the frames that fail the CRC or are deferred to
    // tx_rows (the retry and exact decodes read those), and the uncoded BPSK baseline of the same
    // payloads (channel_kernel's phase A) as per-wavefront partials tx_upart, like cpart
    int tx;
    uint32_t tx_k0, tx_k1;
    int tx_kp, tx_crc_deg;
    int64_t tx_frame0;
    double tx_sigma, tx_scale, tx_unc_sigma;
    const uint32_t* tx_crctab;   // [ceil(kp / 8)][256] CRC remainder of each payload byte value
    const uint64_t* tx_xtab;     // [ceil(K / 8)][256][2] codeword of each message byte value
    double* tx_rows;             // [B][N]
    uint64_t* tx_msg;            // [B][W]
    int32_t* tx_upart;           // [slots][4] (frame, bit errors, 0, 0) of the uncoded baseline, or null
    int64_t* tx_unc_counters;    // its counters (the frame count is added here)
    // fused post pass (scl_lane_kernel FS, PSCL_TUNE_DL_FUSED_POST): a screened retry
    // round's kernel runs dl_post_kernel's work for its own entries after decoding them -- bookkeeping,
    // the CRC stop rule, the replay of the best path, the next flip and its warm state -- and files
    // the survivors in fp.out_list; fp holds the post pass's state arrays exactly as for
    // dl_post_kernel.  Warm-start metrics are then the screening tail's (a screened decode's own);
    // entries the round defers go to bucket 0 of the side list (their exact decode starts at phase 0).
    int fpost;
    pscl_post_params fp;
    const float* fp_beta32g;     // beta in fp32, [K][G][K / G] (lane p's candidates p + G i contiguous), or null
    // 1: an exact decode of the compiled-in N = 128 codes at L = 4, 8 may run on the exact lane-per-path
    // instance (pscl_lane_exact_available: the deferred frames' re-decode, exact forced-bit retry rounds)
    int lane_exact;
    // 1: a screened retry round whose warm-start metrics are screening sums (PSCL_TUNE_DL_WARM_APX):
    // the entries it defers go to bucket 0 of the side list (their exact decode starts at phase 0)
    int warm_apx;
};

#define PSCL_DL_NSEG 8     // 16-phase segments of N = 128: warm-start buckets
#define PSCL_DL_CSTRIDE 16 // int32 stride of the bucket counters (one 64-byte line each)
#define PSCL_DL_DEFERRED 0xFF  /* flags of a retry entry the screening decode deferred (no valid flags value) */

// frame index i of a bucket-list launch -> entry id (pre: bucket prefix counts, pre[0] = 0)
__device__ __forceinline__ int pscl_bucket_of(int64_t i, const int* pre) {
    int k = 0;
#pragma unroll
    for (int q = 1; q < PSCL_DL_NSEG; ++q) k += i >= pre[q] ? 1 : 0;
    return k;
}
__device__ __forceinline__ int64_t pscl_elist_entry(const pscl_decode_params& P, int64_t i, const int* pre) {
    const int k = pscl_bucket_of(i, pre);
    return P.elist[(int64_t)k * P.bcap + (i - pre[k])];
}
// prefix counts of the buckets (wave-uniform loads); returns the total
__device__ __forceinline__ int64_t pscl_bucket_prefix(const int32_t* bcount, int64_t cap, int* pre) {
    int acc = 0;
    pre[0] = 0;
#pragma unroll
    for (int k = 0; k < PSCL_DL_NSEG; ++k) {
        const int c = bcount[k * PSCL_DL_CSTRIDE];
        acc += c < cap ? c : (int)cap;
        pre[k + 1] = acc;
    }
    return acc;
}

// Decision-LLR replay (dlscl.hip): leaf LLRs of a known path, recomputed top-down
struct pscl_replay_params {
    const double* llr;           // channel LLRs [.][N] (or [.][E] with rate matching)
    int N, n, K, W, rm_E;
    const int32_t* rm_src;
    uint64_t info_mask[2];
    const int32_t* count;        // live entries (device)
    const int32_t* list;         // [count] entry ids, or null (entry = position)
    const int64_t* act;          // [entries] LLR row of each entry
    const uint64_t* bits;        // info bits, [.][W] words
    int bits_by_row;             // 1: bits row = act[entry]; 0: bits row = list position
    double* out;                 // [entries][K] decision LLRs (signed), row = entry
};

// DL-SCL post pass of the long codes (N > PSCL_FAST_N, dlscl.hip dl_post_long_kernel): the
// retry decodes run the HIST long kernel, whose best-path decision LLRs are the attempt's L0;
// survivors are compacted into the next round's dense state (no buckets, no warm start).
struct pscl_post_long_params {
    int K, W, rounds, init;
    int64_t cap;                 // entries the state arrays hold
    const int32_t* in_count;     // [1] entries of this pass
    int32_t* out_count;          // [1] entries of the next pass (zeroed before the pass)
    const int64_t* act_in;       // [cap] frame of each entry
    int64_t* act_out;
    const uint64_t* tried_in;    // [cap][W] tried flip indices (null at init: none)
    uint64_t* tried_w_out;
    const int32_t* nt_in;        // [cap] flips tried (null at init)
    int32_t* nt_out;
    const uint64_t* ob;          // [cap][W] the attempt's best bits, by entry
    const uint8_t* of;           // [cap] its flags
    const double* l0;            // [cap][K] its best path's decision LLRs
    uint64_t* force;             // [cap][2W] force words of the next pass, by new entry
    const double* beta;          // [K][K] or null (q = |L0|)
    uint64_t* best;              // [B][W] final best bits (per frame)
    uint8_t* flags;              // [B]
    int32_t* attempts;           // [B] or null
    int32_t* tried_out;          // [B][tried_stride] or null
    int tried_stride;
    int64_t* counters;           // or null: PSCL_CNT_RETRIES += decodes
};

struct pscl_channel_params {
    uint64_t seed;
    uint32_t stream_id;
    int N, K, W, k_payload, crc_deg;
    const uint64_t* xtab;        // [ceil(K/8)][256][2]: codeword x of message byte k = v (linear)
    const uint32_t* crctab;      // [ceil(k_payload/8)][256]: CRC remainder of payload byte k = v
    double sigma, noise_var;
    double llr_scale;            // 2 / noise_var: LLR = (symbol + sigma z) * llr_scale
    double unc_sigma;            // uncoded baseline (run_fer_sweep.py:111-121): its noise sigma (R = 1)
    int64_t* unc_counters;       // [PSCL_NCOUNT] or null: count the uncoded baseline in the same launch
    int64_t frame0, B;
    double* llr;                 // [B][N] (or [B][E] with rate matching)
    uint64_t* msg;               // [B][W] or null
    int rm_E;                    // NR: transmit E symbols, symbol p = x[rm_order[p % N]]
    const int32_t* rm_order;     // [N] sub-block interleaver order
};

int pscl_decode_lmax(int L);
// scl_long.hip (N = 256 .. 1024)
int64_t pscl_long_block_bytes(int N, int L, int K, int hist);
int64_t pscl_long_grid(int64_t B, int L);
hipError_t pscl_launch_long(const pscl_decode_params& P, int hist, hipStream_t s);
// fills P.a_bytes / P.wave_bytes / P.fast for the kernel that will decode this shape
void pscl_decode_layout(pscl_decode_params& P, int hist);
int pscl_fast128_fstride(int L, int ch);
int pscl_screening_available(const pscl_decode_params& P);  // scl128.hip
// lane-per-path screening decoder (scl128_lane.hip): (128,64), L = 8, plain decodes; PSCL_LANE = 0
// builds time scl128_kernel's screening instance instead
#ifndef PSCL_LANE
#define PSCL_LANE 1
#endif
#ifndef PSCL_LANE_NR
#define PSCL_LANE_NR 1
#endif
// screened DL-SCL retry decodes of the (128,64) code on the lane-per-path kernel (1) or the
// two-lanes-per-path forced-bit screening instance (0)
#ifndef PSCL_LANE_FS
#define PSCL_LANE_FS 1
#endif
#ifndef PSCL_LANE4
#define PSCL_LANE4 1
#endif
int pscl_lane_available(const pscl_decode_params& P);
int pscl_lane_frames_per_wg(int L);
hipError_t pscl_launch_lane(const pscl_decode_params& P, int64_t grid, hipStream_t s);
// workgroups of a decode that adds its error counts with atomics (P.ref without P.cpart): each
// wavefront strides over frames and adds its counts once at the end (lane-per-path kernels; the
// two-lanes-per-path kernels' workgroups hold up to PSCL_MAX_WAVES_PER_WG wavefronts)
#ifndef PSCL_LANE_COUNT_GRID
#define PSCL_LANE_COUNT_GRID 32768
#endif
#ifndef PSCL_COUNT_GRID
#define PSCL_COUNT_GRID 8192
#endif
// wavefront slots of the launch pscl_launch_decode makes for P (grid x wavefronts per workgroup)
// when its kernel can store per-wavefront counts (P.cpart), else 0
int64_t pscl_decode_count_slots(const pscl_decode_params& P, int hist);
// counters[FRAME_ERR, BIT_ERR, PAYLOAD_ERR, PAYLOAD_BIT] += the sums of cpart[slots][4], which it
// leaves zero (the kernels store only the slots of wavefronts with errors)
hipError_t pscl_launch_count_reduce(int32_t* cpart, int64_t slots, int64_t* counters, hipStream_t s);
// the DL-SCL baseline decode's screening kernel at N = 128 (PSCL_TUNE_DL_LANE default): 1 the
// lane-per-path kernel, 2 the two-lanes-per-path one, 0 by list size (lane-per-path at L = 8).
// 1: with the lighter retry chains of round 4 (screened lane-per-path retry decodes, side chain,
// fp32 beta in LDS) the lane kernel wins at L = 4 too (config 4: 2.86-2.91 against 3.08-3.09 ms,
// profiles/r04k2_dl_knobs.txt)
#ifndef PSCL_DL_LANE_DEFAULT
#define PSCL_DL_LANE_DEFAULT 1
#endif
// scl_lane_long.hip: the lane-per-path screening decoder of the long codes (N = 256..1024, L = 4, 8)
int pscl_lane_long_available(const pscl_decode_params& P);
// an N = 128 screening launch that runs it (codes without a compiled-in screening kernel)
int pscl_lane_long128_available(const pscl_decode_params& P);
hipError_t pscl_launch_lane_long(const pscl_decode_params& P, hipStream_t s);
int64_t pscl_lane_long_grid(const pscl_decode_params& P);
int pscl_screening_fs_available(const pscl_decode_params& P);  // forced-bit screening (DL-SCL retries)
// the lane-per-path form of a screened DL-SCL retry decode (scl128_lane.hip, FS)
int pscl_lane_fs_available(const pscl_decode_params& P);
hipError_t pscl_launch_lane_fs(const pscl_decode_params& P, int64_t grid, hipStream_t s);
int pscl_lane_exact_available(const pscl_decode_params& P);
hipError_t pscl_launch_lane_exact(const pscl_decode_params& P, hipStream_t s);
int64_t pscl_lane_exact_grid(const pscl_decode_params& P);  // its workgroups (one wavefront each)
hipError_t pscl_launch_decode128(const pscl_decode_params& P, int hist, int wpg, int64_t grid, int lds, hipStream_t s);
int64_t pscl_decode_grid(const pscl_decode_params& P);
int pscl_decode_wpg(const pscl_decode_params& P);
int pscl_decode_lds(const pscl_decode_params& P, int hist);
hipError_t pscl_launch_decode(const pscl_decode_params& P, int hist, hipStream_t s);
hipError_t pscl_launch_channel(const pscl_channel_params& P, hipStream_t s);
// fused TX: channel_kernel's rows of the listed frames (list[0, min(*count, cap)), frame counter
// frame0 + list[i], row rows + 128 list[i]); P carries the tx_* stream parameters
hipError_t pscl_launch_tx_rows(const pscl_decode_params& P, const int64_t* list, const int32_t* count, int64_t cap,
                               double* rows, int64_t frame0, hipStream_t s);
hipError_t pscl_launch_uncoded(const pscl_channel_params& P, int64_t* counters, hipStream_t s);
hipError_t pscl_launch_dl_compact(const uint8_t* flags, int64_t B, int64_t base, int64_t* act, int32_t* list,
                                  int32_t* count, hipStream_t s);
hipError_t pscl_launch_iota64(int64_t* out, int64_t n, hipStream_t s);
hipError_t pscl_launch_replay(const pscl_replay_params& R, int64_t cap, hipStream_t s);
hipError_t pscl_launch_tail_abs_scan(uint32_t lo, uint32_t hi, const uint64_t* exp_table, unsigned long long* out,
                                     hipStream_t s, int bits);
hipError_t pscl_launch_softplus_tails(const double* v, int64_t n, const uint64_t* exp_table, double* exact,
                                     double* apx, hipStream_t s);
hipError_t pscl_launch_dl_post(const pscl_post_params& Q, int64_t entries, hipStream_t s);
int pscl_post_epw(const pscl_post_params& Q);  // entries per wavefront the launch runs with
hipError_t pscl_launch_dl_post_long(const pscl_post_long_params& Q, hipStream_t s);
hipError_t pscl_launch_dl_count(const uint64_t* best, const uint8_t* flags, const uint64_t* ref, int64_t B, int W,
                                int k_payload, int64_t* counters, hipStream_t s);

#endif
