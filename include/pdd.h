/*
 * pdd.h — C ABI of libpdd.so, the MI355X (gfx950) incoherent-dedispersion
 * engine behind pypulsar's `Spectra` hot path.
 *
 * Conventions:
 *   - every entry point returns int status: 0 = ok, < 0 = error;
 *     pdd_last_error() returns a thread-local message for the last failure;
 *   - all array pointers are DEVICE pointers owned by the caller (torch
 *     tensors or any hipMalloc'd memory) unless the name says `host_`;
 *     the library never frees caller memory;
 *   - every compute call takes a hipStream_t (passed as void*) and is
 *     asynchronous on it; pdd_sync() is the only synchronisation;
 *   - 2-D arrays are row-major with an explicit leading dimension `ld`
 *     (elements between consecutive rows);
 *   - the delay-bin tables are built on the host in float64 (bit-exact with
 *     the reference) and passed in as int32.
 *
 * Each entry point cites the reference interface it replaces (file:line in
 * emilieparent/pypulsar).
 */
#ifndef PDD_H
#define PDD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* element types */
enum { PDD_F32 = 0, PDD_U8 = 1, PDD_U16 = 2 };
/* pad modes (Spectra.shift_channels padval, formats/spectra.py:81-94) */
enum {
  PDD_PAD_VALUE = 0,  /* per-channel pad value from `padvals` (number / 'mean' / 'median') */
  PDD_PAD_ROTATE = 1  /* psr_utils.rotate wrap-around (padval == 'rotate') */
};
/* channel statistics: pad values for 'mean'/'median' (spectra.py:83-86);
 * std (population, float64 two-pass), min, max for scaled/scaled2
 * (spectra.py:140-188) */
enum { PDD_STAT_MEAN = 0, PDD_STAT_MEDIAN = 1, PDD_STAT_STD = 2, PDD_STAT_MIN = 3, PDD_STAT_MAX = 4 };
/* zero-DM layouts */
enum { PDD_LAYOUT_TIME_MAJOR = 0, /* [nspec][nchan], filterbank file order */
       PDD_LAYOUT_CHAN_MAJOR = 1  /* [nchan][nspec], Spectra.data order    */ };

int pdd_version(void);
const char* pdd_last_error(void);
/* Identity of this build: the 16-hex-digit digest of the HIP sources and
 * compile flags the library was built from (pypulsar_amd/_digest.py computes
 * the same from a source tree).  The Python host refuses a library whose
 * digest differs from its sources, and profiling evidence is stamped with it,
 * so counters are only reported for the binary that produced them. */
const char* pdd_source_digest(void);
/* Free the device scratch the library keeps per (device, stream, calling host
 * thread) -- sweep images, partial sums; synchronises the device.  Optional:
 * the next call that needs scratch allocates it again.  Scratch is keyed by
 * the calling thread, so several host threads may queue work on one stream
 * (each gets its own buffers, e.g. an 8 GiB sweep image each); a thread's
 * buffers stay allocated after it exits until this call.  Returns the first
 * HIP error (every buffer is still freed). */
int pdd_scratch_release(void);
/* hipStreamSynchronize(stream) */
int pdd_sync(void* stream);

/* Corner turn [nspec][nchan] (in_dtype) -> [nchan][nspec] (out_dtype: PDD_F32,
 * or the input dtype for a raw byte transpose).
 * Replaces filterbank.get_spectra's reshape + `.T` + Spectra.__init__'s
 * astype('float') (formats/filterbank.py:153-157, formats/spectra.py:34) and
 * mockspecfil2subbands' per-block transpose (bin/mockspecfil2subbands.py:155-175). */
int pdd_corner_turn(const void* in, int in_dtype, int64_t nspec, int64_t nchan, int64_t ld_in,
                    void* out, int out_dtype, int64_t ld_out, void* stream);

/* Elementwise dtype conversion of a [rows][cols] array to float32
 * (Spectra.__init__ data.astype, formats/spectra.py:34, for C-ordered input). */
int pdd_convert_f32(const void* in, int in_dtype, int64_t rows, int64_t cols, int64_t ld_in,
                    float* out, int64_t ld_out, void* stream);

/* Per-channel statistic of x[C][N] -> out[C] (float32): mean / median (pad
 * values of Spectra.shift_channels 'mean'/'median', formats/spectra.py:83-86;
 * Spectra.masked maskvals, spectra.py:216-222), std / min / max
 * (Spectra.scaled / scaled2 per-channel terms, spectra.py:157-187). */
int pdd_channel_stats(const float* x, int64_t C, int64_t N, int64_t ld, int stat,
                      float* out, void* stream);

/* out[c][t] = X(c, t + bins[c]) for t < n_out, X = x inside [0,N), padvals[c]
 * (PDD_PAD_VALUE) or wrap (PDD_PAD_ROTATE) outside.
 * Replaces Spectra.shift_channels (formats/spectra.py:54-94) incl.
 * psr_utils.rotate (spectra.py:80). `out` must not alias `x`. */
int pdd_shift_pad(const float* x, int64_t C, int64_t N, int64_t ld, const int32_t* bins,
                  int pad_mode, const float* padvals, float* out, int64_t ld_out,
                  int64_t n_out, void* stream);

/* Fused shift + group sum: out[k][t] = sum_{c in group k} X(c, t + bins[c]),
 * groups = nsub contiguous blocks of C/nsub channels, t < n_out.
 * nsub == nchan-groups: Spectra.subband (formats/spectra.py:96-138);
 * nsub == 1: Spectra.dedisperse + channel sum, the dedispersed series of
 * bin/waterfaller.py:140 (spectra.py:229-260).  bins may be NULL (no shift). */
int pdd_shift_group_sum(const float* x, int64_t C, int64_t N, int64_t ld, const int32_t* bins,
                        int pad_mode, const float* padvals, int64_t nsub, float* out,
                        int64_t ld_out, int64_t n_out, void* stream);

/* out[c][j] = sum_{k<factor} x[c][j*factor + k], j < N/factor.
 * Replaces Spectra.downsample (formats/spectra.py:329-351). */
int pdd_downsample(const float* x, int64_t C, int64_t N, int64_t ld, int64_t factor,
                   float* out, int64_t ld_out, void* stream);
/* The same on 8-bit channel rows (a Spectra's unmodified raw bytes): exact
 * integer sums, written as float32; reads a quarter of the float32 image's
 * bytes.  Used by the DDplan executor (spectra.py:329-351 per DDstep). */
int pdd_downsample_u8(const uint8_t* x, int64_t C, int64_t N, int64_t ld, int64_t factor,
                      float* out, int64_t ld_out, void* stream);
/* The same co-add kept as uint16 (factor 1..4: sums <= 1020), the input of
 * the exact 16-bit sweep (PDD_U16) -- the DDplan executor's downsampled
 * 8-bit steps (formats/spectra.py:329-351 on raw 8-bit rows). */
int pdd_downsample_u8_u16(const uint8_t* x, int64_t C, int64_t N, int64_t ld, int64_t factor,
                          uint16_t* out, int64_t ld_out, void* stream);

/* Zero-DM filter: every spectrum minus its channel mean; integer data use
 * round-half-even of the float64 mean and wrap modulo 2^nbits, float32 data
 * stay float32.  Replaces bin/zero_dm_filter.py:30-50 (filter + write loop).
 * `out` may alias `in`. */
int pdd_zero_dm(const void* in, int dtype, int64_t nspec, int64_t nchan, int64_t ld,
                int layout, void* out, int64_t ld_out, void* stream);

/* Streaming prologue, one HBM pass over a time-major block [nspec][nchan]
 * (filterbank order, u8/u16/f32): corner turn + zero-DM in float mode
 * (zero_dm != 0: every spectrum minus its float64 channel mean, the
 * subtraction of bin/zero_dm_filter.py:30-39 without the integer cast) +
 * Spectra.downsample(factor) (formats/spectra.py:329-351; factor divides 64):
 *   out[c][j] = sum_{k<factor} (x[j*factor+k][c] - mean[j*factor+k]),
 * j < nspec / factor, out channel-major float32. */
int pdd_zdm_downsample(const void* in, int dtype, int64_t nspec, int64_t nchan, int64_t ld,
                       int64_t factor, int zero_dm, float* out, int64_t ld_out, void* stream);

/* The 8-bit prologue of the exact 16-bit sweep (streaming configs[4]): the
 * same zero-DM + downsample + corner turn in integer arithmetic,
 *   out[c][j] = offset + sum_{k<factor} z(x[j*factor+k][c]),  uint16, channel-major,
 * with m = the spectrum's channel mean rounded half-to-even (np.round, as
 * bin/zero_dm_filter.py:30-39) and z by mode:
 *   PDD_ZDM_NONE  z = x                  (no filter; plain downsample)
 *   PDD_ZDM_INT   z = x - m, signed      (integer zero-DM without the uint8 wrap)
 *   PDD_ZDM_WRAP  z = (x - m) mod 256    (the reference's uint8 result exactly)
 * 8-bit input with 16-byte-aligned rows (nchan % 16 == 0); offset must keep
 * every value in [0, 65535] (PDD_ZDM_INT: offset >= 255 factor).  For the
 * 16-bit sweep (values <= 1023): factor <= 2 for PDD_ZDM_INT (offset 255
 * factor), <= 4 otherwise (offset 0). */
enum { PDD_ZDM_NONE = 0, PDD_ZDM_INT = 1, PDD_ZDM_WRAP = 2 };
int pdd_zdm_int_downsample(const void* in, int dtype, int64_t nspec, int64_t nchan, int64_t ld,
                           int64_t factor, int mode, int offset, uint16_t* out, int64_t ld_out,
                           void* stream);

/* ---- waterfaller post-chain (Spectra.scaled / scaled2 / masked / smooth) ---- */
/* Whole-array statistics of x[C][N] into out4 (device float[4]):
 * {mean, population std, min, max}, float64 accumulation.
 * Replaces other.data.std() / other.data.max() (formats/spectra.py:156, 181). */
int pdd_global_stats(const float* x, int64_t C, int64_t N, int64_t ld, float* out4, void* stream);
/* out[c][t] = (x[c][t] - sub[c*sub_inc]) / div[c*div_inc] (inc 0 = broadcast).
 * Replaces the per-channel loops of Spectra.scaled (formats/spectra.py:157-162)
 * and Spectra.scaled2 (spectra.py:182-187). */
int pdd_scale_rows(const float* x, int64_t C, int64_t N, int64_t ld, const float* sub,
                   int64_t sub_inc, const float* div, int64_t div_inc, float* out, int64_t ld_out,
                   void* stream);
/* out[c][t] = mask[c][t] ? vals[c] : x[c][t]  (mask: uint8 0/1).
 * Replaces np.where(mask, maskvals, data) of Spectra.masked (formats/spectra.py:225-226). */
int pdd_masked_fill(const float* x, int64_t C, int64_t N, int64_t ld, const uint8_t* mask,
                    int64_t ld_mask, const float* vals, float* out, int64_t ld_out, void* stream);
/* Boxcar of `width` samples and height 1/sqrt(width), 'same' centring, per
 * channel, padded with padvals[c] (PDD_PAD_VALUE: number / 'mean' / 'median')
 * or wrapped (PDD_PAD_ROTATE: 'wrap').  Replaces Spectra.smooth
 * (formats/spectra.py:262-303; scipy.signal.convolve). `out` must not alias x. */
int pdd_smooth(const float* x, int64_t C, int64_t N, int64_t ld, int64_t width, int pad_mode,
               const float* padvals, float* out, int64_t ld_out, void* stream);

/* ---- batched DM sweep (new executor over utils/DDplan2b.py grids) ----
 * plane[d][t] = sum_c X(c, t + table[d][c]), t < n_out (defaults of
 * Spectra.dedisperse(dm, padval, trim=True) + channel sum, per DM trial,
 * formats/spectra.py:229-260 + bin/waterfaller.py:140).
 * The plan holds the device copy of the delay table and its per-block
 * extents; it is built once per (grid, channel count, dtype). */
typedef struct pdd_sweep_plan pdd_sweep_plan;

/* host_table: [D][C] int32, row d = the bins Spectra.dedisperse(dms[d])
 * would pass to shift_channels.  dtype: PDD_F32, PDD_U8 or PDD_U16 (samples
 * <= 1023) input. */
int pdd_sweep_plan_create(const int32_t* host_table, int64_t D, int64_t C, int dtype,
                          pdd_sweep_plan** plan);
/* The same with plan flags (pdd_sweep_plan_create = PDD_SWEEP_FACTOR):
 * PDD_SWEEP_FACTOR lets a single-group plan sweep factorised over groups of
 * 4 (or 2) adjacent channels when the plan's cost model says it pays: each
 * group's distinct relative-shift patterns are summed once (stage 1), and
 * every trial adds its pattern series at the group's base shift (stage 2).
 * Integer plans (PDD_U8 / PDD_U16, also through pdd_sweep_execute_ds) sum
 * the same integer samples as the channel-by-channel kernel: the plane is
 * bit-identical.  PDD_F32 plans regroup the float32 channel sum (within the
 * float32 bar; exact for integer-valued data).  Flags 0 forces the
 * channel-by-channel kernel.  Factorised plans take the plain and the
 * pieces layouts and column offsets; they do not chain
 * (pdd_subband_chain). */
#define PDD_SWEEP_FACTOR 1
/* with PDD_SWEEP_FACTOR: factorise whenever the windows fit, paying or not
 * (tests of small grids) */
#define PDD_SWEEP_FACTOR_FORCE 2
/* with PDD_SWEEP_FACTOR: groups of 2 channels only (default: 4 or 2, the
 * cheaper by the plan's cost model; 2 where a 4-channel group's pattern
 * windows do not fit one LDS chunk buffer) */
#define PDD_SWEEP_FACTOR_G2 4
#define PDD_SWEEP_FACTOR_G4 8  /* groups of 4 channels only */
/* with PDD_SWEEP_FACTOR: plane-aligned factorised tiles (default: each trial's
 * time tile is skewed by its delay at a mid-band reference group, so a
 * tile's pattern windows span less drift; the plane is identical) */
#define PDD_SWEEP_NO_SKEW 16
int pdd_sweep_plan_create_ex(const int32_t* host_table, int64_t D, int64_t C, int dtype, int flags,
                             pdd_sweep_plan** plan);
/* Channels per factor group of the plan (4 or 2; 0 = channel by channel) and, if
 * n_patterns is non-null, its stage-1 pattern count. */
int pdd_sweep_plan_factor(const pdd_sweep_plan* plan, int64_t* n_patterns);
/* Largest per-trial time-tile skew of a factorised plan's delay-aligned tiles
 * (samples of an eighth / quarter; 0: plane-aligned tiles or a channel plan),
 * and, if extra_tiles is non-null, the time tiles each segment adds for it. */
int pdd_sweep_plan_skew(const pdd_sweep_plan* plan, int64_t* extra_tiles);
/* x: [C][N] (ld) of the plan's dtype; out: [D][ld_out] float32.
 * For PDD_U8 with PDD_PAD_VALUE every padvals[c] must be an integer in
 * [0, 255] (checked on the host side by the caller).  PDD_U16 input: unsigned
 * 16-bit samples <= 1023 (e.g. the offset output of pdd_zdm_int_downsample),
 * swept exactly with the packed-u16 kernels. */
int pdd_sweep_execute(const pdd_sweep_plan* plan, const void* x, int64_t N, int64_t ld,
                      int pad_mode, const float* padvals, float* out, int64_t ld_out,
                      int64_t n_out, void* stream);
/* The same with two more input layouts/offsets (DM-sharded sweeps):
 *   piece == 0: x is channel-major [C][ld];
 *   piece == P > 0 (a power of two): x is [ceil(N/P)][C][P] -- the block an
 *     all-gather of per-rank channel-major time slices of P samples produces
 *     (sample s of channel c at x[(s/P)*C*P + c*P + s%P]);
 *   x_off: plane column t sums input samples t + x_off + table[d][c] (a column
 *     range [x_off, x_off + n_out) of the full sweep); pads apply outside
 *     [0, N) of x;
 *   out_bias: added to every plane value (e.g. -offset * C for offset input). 
 * Offsets and pieces need the interleaved tilings (every grid whose shift
 * span per trial block fits the LDS); sparser grids return an error. */
int pdd_sweep_execute_ex(const pdd_sweep_plan* plan, const void* x, int64_t N, int64_t ld,
                         int64_t piece, int64_t x_off, int pad_mode, const float* padvals,
                         float* out, int64_t ld_out, int64_t n_out, float out_bias,
                         void* stream);
/* Staged execution of a factorised plan (pdd_sweep_plan_factor > 0, raw-rate
 * input) for pipelining: stage 1 (1: the pattern image, written into
 * `patterns`), stage 2 (2: the sweep, reading the pattern image stage 1 of the
 * same x / x_off / n_out wrote into `patterns`) or both (3), one segment (the
 * whole column range) per call, arguments as pdd_sweep_execute_ex.  Two
 * pattern buffers let stage 1 of the next block run on one stream while
 * stage 2 of this block runs on another (DMShardedSweep: CU-partitioned
 * streams, pdd_stream_create_cu_mask).  `pattern_bytes` must be >=
 * pdd_sweep_pattern_bytes(plan, n_out). */
int64_t pdd_sweep_pattern_bytes(const pdd_sweep_plan* plan, int64_t n_out);
int pdd_sweep_execute_stage(const pdd_sweep_plan* plan, const void* x, int64_t N, int64_t ld,
                            int64_t piece, int64_t x_off, int pad_mode, const float* padvals,
                            float* out, int64_t ld_out, int64_t n_out, float out_bias,
                            void* patterns, int64_t pattern_bytes, int stage, void* stream);
/* A stream whose kernels run only on the CUs set in `mask` (n_words 32-bit
 * words, bit i = CU i; hipExtStreamCreateWithCUMask) / its release. */
int pdd_stream_create_cu_mask(const uint32_t* mask, int n_words, void** stream);
int pdd_stream_destroy(void* stream);
/* Grouped sweep: n_grp independent channel groups of C channels each
 * (channels g*C .. g*C+C-1 of the input), every group with its own [D][C]
 * table: host_table is [n_grp][D][C].  One launch replaces n_grp sweeps --
 * the stage-1 subband passes of a DDplan step (Spectra.subband at each subDM,
 * formats/spectra.py:96-138, one group per subband) or the stage-2 sweeps of
 * its passes (one group per pass).  Trial d of group g is written to plane
 * row g*row_g + d*row_d. */
int pdd_sweep_plan_create_grouped(const int32_t* host_table, int64_t n_grp, int64_t D, int64_t C,
                                  int dtype, pdd_sweep_plan** plan);
int pdd_sweep_execute_grouped(const pdd_sweep_plan* plan, const void* x, int64_t N, int64_t ld,
                              int pad_mode, const float* padvals, float* out, int64_t ld_out,
                              int64_t n_out, int64_t row_g, int64_t row_d, void* stream);
/* Sweep of an 8-bit block downsampled by ds (2..4) on the fly: x8 is
 * channel-major [C_all][ld] uint8 at the raw rate (n_raw samples); the swept
 * series is Spectra.downsample(ds) of it (formats/spectra.py:329-351: N =
 * n_raw / ds co-adds, exact integers <= 1020), so the plan must be PDD_U16.
 * Grouped and ungrouped plans (ungrouped: row_g 0, row_d 1); pads act on the
 * downsampled series (integers <= 1023 or PDD_PAD_ROTATE).  Replaces
 * pdd_downsample_u8_u16 + pdd_sweep_execute(_grouped) of a DDplan step
 * (utils/DDplan2b.py:102-199 downsamp) without the downsampled copy. */
int pdd_sweep_execute_ds(const pdd_sweep_plan* plan, const uint8_t* x8, int64_t n_raw, int64_t ld,
                         int64_t ds, int pad_mode, const float* padvals, float* out,
                         int64_t ld_out, int64_t n_out, int64_t row_g, int64_t row_d,
                         void* stream);
/* Both stages of a subbanded DDplan step in two launches and no subband
 * plane: stage 1 (plan1: grouped, one group per subband, trials = the passes'
 * subDMs; PDD_U8 rows at ds 1 or PDD_U16 with x = 8-bit rows co-added by
 * ds 2..4 on the fly, as pdd_sweep_execute_ds) writes its rows -- trial d of
 * group g = stage-2 channel d * n_grp1 + g, i.e. the subbands of pass d --
 * directly as stage 2's float32 quarters image; stage 2 (plan2: PDD_F32,
 * grouped, one group per pass, delays >= 0) sweeps that image into out (trial
 * d of group g at row g*row_g + d*row_d, n_out columns).  pad2vals[c]: the
 * value pad of stage-2 channel c (Spectra.dedisperse padval on the subbanded
 * data).  Equals pdd_sweep_execute(_grouped/_ds) of stage 1 into a
 * [n_grp2*C2][N1] subband plane followed by pdd_sweep_execute_grouped of
 * stage 2 over it (formats/spectra.py:96-138 then :229-260 per pass).
 * Returns PDD_ENOCHAIN (-5), with nothing launched, for a block/grid it
 * cannot chain (a stage that needs more than one segment, or a stage-2 delay
 * span wider than an eighth of the block): run the two stages apart then.
 * Any other negative status (e.g. -2: scratch allocation failed) is an
 * error of this call. */
#define PDD_ENOCHAIN (-5)
int pdd_subband_chain(const pdd_sweep_plan* plan1, const void* x, int64_t n_raw, int64_t ld,
                      int64_t ds, int pad1_mode, const float* pad1vals,
                      const pdd_sweep_plan* plan2, const float* pad2vals, float* out,
                      int64_t ld_out, int64_t n_out, int64_t row_g, int64_t row_d, void* stream);
/* Extents used by the plan (for DESIGN/bench reporting): DM trials, channels,
 * DMs per block, time samples per block, LDS bytes per workgroup. */
int pdd_sweep_plan_info(const pdd_sweep_plan* plan, int64_t* info /*[8]*/);
/* Integer-input plans (PDD_U8, PDD_U16): the largest sample value the
 * caller's input (and integer pads) can hold, default 255 / 1023.  The
 * sweep adds two samples per 32-bit lane pair and converts every
 * floor(65535 / max_value) channels (at most 256), so a tighter bound means
 * fewer conversions; a sample above it gives wrong sums.  E.g. the
 * zero_dm_filter.py:30-39 uint8-wrap image co-added by 2 is <= 510. */
int pdd_sweep_plan_set_input_max(pdd_sweep_plan* plan, int max_value);
/* Test switches of a plan (parity tests and the C-ABI driver; both default
 * off).  poison: factorised plans fill their pattern image with 0xFF bytes
 * before stage 1 of every segment, so a stage-2 read of an element stage 1
 * did not write shows as a NaN / overflowed lane.  segment_bytes > 0: the
 * scratch budget of one time segment (default: 16 GiB, 80 GiB for factorised
 * plans, capped by free device memory), to run the multi-segment path on
 * small blocks. */
int pdd_sweep_plan_set_poison(pdd_sweep_plan* plan, int on);
int pdd_sweep_plan_set_segment_bytes(pdd_sweep_plan* plan, int64_t bytes);
int pdd_sweep_plan_destroy(pdd_sweep_plan* plan);
/* Measurement hooks (bench.py): with timing on, every sweep-kernel launch
 * of pdd_sweep_execute(_grouped) -- not the interleave pre-pass -- is
 * bracketed by its own pair of HIP events on the execute stream (no host
 * synchronisation; up to 1024 launches between reads).
 * pdd_sweep_timing_read waits for the last one and returns the SUM of the
 * bracketed durations and the number of launches since the previous read;
 * pdd_sweep_kernel_ms is the same sum alone. */
int pdd_sweep_set_timing(pdd_sweep_plan* plan, int on);
int pdd_sweep_timing_read(pdd_sweep_plan* plan, float* total_ms, int64_t* launches);
int pdd_sweep_kernel_ms(pdd_sweep_plan* plan, float* ms);

/* ---- single-pulse boxcar search over a DM-time plane (SURVEY.md §8(f)
 * rank 4; no reference search -- the boxcar is Pulse.smooth,
 * formats/pulse.py:217-241; definition in pypulsar_amd/search.py).
 * x: [D][n] float32 plane, row stride ld.  L: detrend chunk length. */
/* Per row and chunk of L samples (last may be short): mean and 1/std
 * (0 where std == 0), written to [D][ceil(n/L)] arrays. */
int pdd_sp_chunk_stats(const float* x, int64_t D, int64_t n, int64_t ld, int64_t L, float* mean,
                       float* istd, void* stream);
/* Boxcar S/N of every start and width (widths: HOST array, ascending,
 * 1..1025, at most 32) on the chunk-normalised rows; one candidate per
 * (row, window of 1024 starts) with S/N >= threshold, appended to cands as
 * int32 records {row, start, width, float-bits snr} through the device
 * counter *count (incremented for every candidate, stored while
 * < max_cands: the caller checks for overflow).  Record order is not
 * deterministic; the set is.
 * Streams: a row may continue into a second plane -- row d is
 * x[d][0:n] followed by x_next[d][0:n_next] (n % L == 0; its chunks use
 * mean_next/istd_next, [D][ceil(n_next/L)]) -- and only starts < n_starts
 * are searched, so block i of a stream is searched with the first columns
 * of block i+1 exactly as the one-shot plane would be.  n_next = 0 (and
 * null next pointers): a single plane. */
int pdd_sp_search(const float* x, int64_t D, int64_t n, int64_t ld, int64_t L, const float* mean,
                  const float* istd, const float* x_next, int64_t n_next, int64_t ld_next,
                  const float* mean_next, const float* istd_next, int64_t n_starts,
                  const int32_t* widths, int n_widths, float threshold, int32_t* cands,
                  int64_t max_cands, unsigned long long* count, void* stream);

/* ---- PSRFITS search-mode subints -> [nchan][N] float32 (SURVEY.md §8(f)
 * rank 3).  Replaces psrfits.unpack_4bit (formats/psrfits.py:37-50),
 * PsrfitsFile.read_subint (:67-107: ((data*scales)+offsets)*weights in
 * float32) and get_spectra (:140-183: concatenation, transpose, skip/trunc,
 * band flip).  raw: nsub consecutive SUBINT table rows as stored (row_bytes
 * each, big-endian; DATA at byte data_off of a row); nbits 4/8/16/32;
 * wso: [nsub][3][nchan] float32 scales, offsets, weights; output row
 * c' = flip ? nchan-1-c : c holds samples s0 .. s0+N-1 of the concatenated
 * subints. */
int pdd_psrfits_subints(const uint8_t* raw, int64_t nsub, int64_t row_bytes, int64_t data_off,
                        int nbits, int64_t nsblk, int64_t nchan, const float* wso, int64_t s0,
                        int64_t N, int flip, float* out, int64_t ld_out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PDD_H */
