/*
 * csmom.h -- C ABI of libcsmom.so, the MI355X (gfx950) engine for the cross-sectional
 * momentum backtest hot path of
 * AkshayJha22/Cross-Sectional-Momentum-Strategy-Replication-Backtesting-Framework.
 *
 * The reference has no FFI: its boundary is plain Python functions on pandas objects
 * (SURVEY.md section 8(b)).  Each entry point below replaces the arithmetic of one of
 * those functions; the Python layer in the package keeps the reference's signatures and
 * calls these through ctypes.
 *
 * Conventions
 *   - Every array argument is a DEVICE pointer (hipMalloc / torch ROCm tensor) unless it
 *     is documented as a host pointer.  Buffers are caller-owned.
 *   - Dense row-major [T][N] layouts, assets fastest, float64 throughout.
 *   - A cell with no daily row ("absent") holds the NaN payload CSM_ABSENT_BITS; a present
 *     row with a missing price holds an ordinary NaN.
 *   - Calls are asynchronous on the context's stream (csm_set_stream); csm_sync waits.
 *   - Every call returns CSM_OK (0) or a negative status; csm_last_error() describes it.
 *   - A context is not thread-safe; separate contexts may be used concurrently.
 */
#ifndef CSMOM_H
#define CSMOM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CSM_ABI_VERSION 3
#define CSM_ABSENT_BITS 0x7FF4000000000001ULL

#define CSM_OK 0
#define CSM_E_INVAL (-1)   /* bad argument (null pointer, size, unsupported parameter) */
#define CSM_E_HIP (-2)     /* HIP runtime / launch failure */
#define CSM_E_RCCL (-3)    /* RCCL missing or a collective failed */
#define CSM_E_TIMEOUT (-4) /* an in-launch hand-off gave up a wait: that launch's outputs are invalid */
#define CSM_UNIQUE_ID_BYTES 128

typedef struct csm_ctx csm_ctx;

int csm_abi_version(void);

/* Process-wide knobs that select between PRODUCT paths with identical results (so tests can
 * drive the fallbacks on inputs that would not reach them): "signal_vec" (2 paired 16-B rows |
 * 1 one asset per lane, the odd-N path), "signal_bwf" (0 auto | 1 one-wave blocks | 4 the wide
 * panels' four barrier-free waves with buffer loads), "signal_j12" (1 the wide date-shard kernel's
 * J = 12 with the product length fixed at compile time | 0 runtime J), "cols_wg" (1 the halo pass's listed
 * columns summarised / repaired one workgroup per column, month prices derived together in LDS |
 * 0 one thread per column), "dec_merge" (1 the merged decile sweep on
 * ids, the general kernel for the rows it leaves | 0 the general kernel only), "dec_split" (2
 * auto: wide rows on ids take the split pass -- plan, chunked sweep, finish -- in launches of
 * fewer rows than half the CUs (short date shards) | 1 always | 0 the merged pass with one
 * workgroup per row; the same labels, counts and means bit for bit), "mj_reg"
 * (csm_momentum_multi: 2 register ring, two assets per lane | 1 one asset | 0 the LDS ring),
 * "dec_narrow_max" (widest row for the narrow-row decile kernels), "cohort_seg" / "cohort_lds"
 * (portfolio cohort-sum kernel: label-sorted segments (rows <= 7168) | per-wave LDS sums |
 * register sums; "cohort_seg" changes the chunk plan, so set it before sizing the portfolio
 * workspace), "turn_want" (turnover workgroups per launch, default 4096; set before sizing
 * the portfolio workspace), "turn_gen_grid" (workgroups of the general-row turnover launch,
 * default 8192), "overlap_rows" (1 one thread per (month, panel, decile) for single-chunk
 * plans | 0 one per (K, month, panel, decile)), "gen_reset" (1 the turnover work-list counter
 * reset by a kernel | 0 by hipMemsetAsync, round 3's form, kept for the graph-replay diagnosis
 * of tests/test_gpu_capture.py), "turn_vwg" (1 a grouped batch's steady value-weight turnover
 * rows by one workgroup per weight panel | 0 one per row), "turn_mask" (1 steady equal-weight
 * legs turnover rows counted from the legs label sort's leg bitplanes | 0 from the label
 * bytes), "ls_opt" (1 the one-wave legs label sort's prefix ranks by v_mbcnt | 0 masked
 * popcounts), "dec_split_cells" (cells per chunk of the split decile sweep, default 32768, a
 * multiple of 8192 -- the merged pass's sweep trip -- so the merged and split passes sum every
 * row's decile means in the same order; the split workspace is the context's), "dec_split_pf"
 * (the split sweep: 0 two workgroups per CU, the default | 1 one prefetching workgroup per CU |
 * 2 the prefetching one when the launch has no more (chunk, date) pairs than CUs; the same
 * bits either way), "tc_spins" (polling trips a
 * csm_signal_chunked workgroup makes before it gives up a wait, default 2^21; 0 gives up at
 * once, which only the tests of the CSM_E_TIMEOUT report set).
 * Returns CSM_E_INVAL for an unknown key or value. */
int csm_tune(const char* key, int value);
/* Profiling aids: "dec_timing" = device int64 buffer [T_m][9] that k_deciles fills with
 * wall-clock ticks (100 MHz) at its phase boundaries; "gen_probe" = device int32 that receives
 * the turnover work-list length the general-row launch read (NULL switches either off). */
int csm_tune_ptr(const char* key, void* p);

/* Create a context bound to HIP device `device` (stream = the null stream). */
int csm_create(int device, csm_ctx** out);
int csm_destroy(csm_ctx* ctx);
const char* csm_last_error(const csm_ctx* ctx);
/* Launch subsequent work on `stream` (a hipStream_t; NULL = the null stream). */
int csm_set_stream(csm_ctx* ctx, void* stream);
int csm_sync(csm_ctx* ctx);

/*
 * Month-end aggregation.  Replaces the `groupby(['ticker', Grouper(freq='ME')])
 * .agg(adj_close=last, monthly_volume=sum)` of src/features.py:34-39.
 *   P[T_d][N]        daily adj_close (ABSENT / NaN encoded)
 *   V[T_d][N]        daily volume, nullable (NaN counts as 0, features.py:31)
 *   month_start[T_m+1] int64 day offsets of each month (device)
 *   PM[T_m][N]       out: last non-NaN price; NaN if the month has rows but no price;
 *                    ABSENT if it has no row
 *   VOL[T_m][N]      out, nullable: pandas-Kahan sum of volume over present days
 */
int csm_month_end(csm_ctx* ctx, const double* P, const double* V, int64_t T_d, int64_t N,
                  const int64_t* month_start, int32_t T_m, double* PM, double* VOL);

/*
 * ret_1m / mom_J / next_ret scan over present rows of each asset.  Replaces
 * src/features.py:44-52 (pct_change with ffill; shift(skip).rolling(J).apply(prod))
 * and run_demo.py:48 (next-row return within the ranked subset).
 *   PM[T_m][N]   month prices from csm_month_end
 *   R, M, NR     out [T_m][N]; R nullable.  NaN where undefined or absent.
 *   carry        nullable [(J+skip)+2][N]: inherited scan state for a date shard
 *                (rows 0..J+skip-1: ring of factors fl(1+ret), oldest first;
 *                row J+skip: pff (last valid price); row J+skip+1: psff)
 *   next_pm      nullable [N]: month price of the first present row after the panel
 *                (ABSENT if none)
 *   carry_out    nullable [(J+skip)+2][N]: scan state after the panel
 * J >= 1, skip >= 0, J + skip <= 256.
 */
int csm_momentum(csm_ctx* ctx, const double* PM, int32_t T_m, int64_t N, int32_t J,
                 int32_t skip, double* R, double* M, double* NR, const double* carry,
                 const double* next_pm, double* carry_out);

/*
 * Several look-backs in one scan (parameter sweeps): Js[nJ] (1 <= nJ <= 4, host array),
 * M[q] / NR[q] host arrays of device [T_m][N] outputs.  One read of PM; each (M[q], NR[q])
 * equals csm_momentum(PM, Js[q], skip) bit for bit.  max(J) + skip <= 64; no carry.
 * Replaces, per sweep batch, the per-J `compute_monthly_momentum_from_daily(...,
 * lookback_months=J)` calls (src/features.py:47-52, run_demo.py:48).
 */
int csm_momentum_multi(csm_ctx* ctx, const double* PM, int32_t T_m, int64_t N,
                       const int32_t* Js, int32_t nJ, int32_t skip, double* const* M,
                       double* const* NR);
/*
 * csm_momentum_multi that also writes, per look-back, ids[q][T_m][N] (uint16, host array of
 * device pointers): each mom_J's fixed-map bucket id (as csm_signal_ids; 0xFFFF = NaN), so the
 * sweep's decile pass (csm_deciles_ids on the [T_m * B][N] rows of a batch) reads 2-B ids and M
 * only near the bin edges.  Same M / NR bits as csm_momentum_multi.
 */
int csm_momentum_multi_ids(csm_ctx* ctx, const double* PM, int32_t T_m, int64_t N,
                           const int32_t* Js, int32_t nJ, int32_t skip, double* const* M,
                           double* const* NR, uint16_t* const* ids);

/*
 * Time-chunked scan for panels with few assets: the months are split into C contiguous
 * chunks that are scanned concurrently from exactly rebuilt boundary states (the date-shard
 * summary/fold of csm_shard_summary / csm_fold_carry, inside one GPU).  Same outputs as
 * csm_momentum (no carry input).  workspace: device buffer of
 * csm_momentum_chunked_workspace(T_m, N, J, skip, C) bytes.
 */
int64_t csm_momentum_chunked_workspace(int32_t T_m, int64_t N, int32_t J, int32_t skip,
                                       int32_t C);
int csm_momentum_chunked(csm_ctx* ctx, const double* PM, int32_t T_m, int64_t N, int32_t J,
                         int32_t skip, int32_t C, double* R, double* M, double* NR,
                         const double* next_pm, void* workspace);
/*
 * csm_momentum_chunked that also writes ids[T_m][N] (uint16): each mom_J's fixed-map bucket id
 * (as csm_signal_ids), so a narrow panel's decile pass (csm_deciles_ids, C2) reads 2-B ids and
 * mom_J only near the bin edges.  Same R / M / NR bits.  N % 4 == 0, 8-B aligned ids.
 */
int csm_momentum_chunked_ids(csm_ctx* ctx, const double* PM, int32_t T_m, int64_t N, int32_t J,
                             int32_t skip, int32_t C, double* R, double* M, double* NR,
                             const double* next_pm, uint16_t* ids, void* workspace);
/*
 * Month-end + time-chunked scan in ONE launch for narrow panels (C2; replaces csm_month_end ->
 * csm_momentum_chunked_ids, four launches): a workgroup reduces one chunk's daily rows of 256
 * assets to month prices in LDS, publishes the chunk's exchange record, folds the records of
 * the earlier chunks of its columns (in-launch hand-off, bounded spins) and scans its months.
 * The same R / M / NR / ids bits as csm_month_end -> csm_momentum (month_start / P as
 * csm_signal; no carry, no next_pm: whole panels).  R and ids nullable.  Even N, months of at
 * most 23 day rows (max_month_days), J + skip <= 32, 1 <= C <= 64 chunks of at most 32
 * months, 16-B aligned P / M / NR / R, 4-B aligned ids.  workspace:
 * csm_signal_chunked_workspace(T_m, N, J, skip, C) bytes, 256-B aligned and ZERO-FILLED before
 * its first use (a launch leaves its sync words zero again; word 2 is set if a wait gave up,
 * which no correct launch does).  One launch at a time per workspace: two launches in flight
 * on different streams must not share one (their tickets and flags would mix).
 * A give-up is never silent: csm_signal_chunked_status reports it.
 */
int64_t csm_signal_chunked_workspace(int32_t T_m, int64_t N, int32_t J, int32_t skip, int32_t C);
int csm_signal_chunked(csm_ctx* ctx, const double* P, int64_t T_d, int64_t N,
                       const int64_t* month_start, int32_t T_m, int32_t max_month_days,
                       int32_t J, int32_t skip, int32_t C, double* R, double* M, double* NR,
                       uint16_t* ids, void* workspace);
/*
 * Synchronises the context's stream and reads the workspace's give-up mark: CSM_OK, or
 * CSM_E_TIMEOUT when a csm_signal_chunked launch on it since the last check gave up a wait (its
 * outputs are invalid); the mark is then cleared.  CSM_E_INVAL while the stream is capturing
 * (check after the graph's replay).
 */
int csm_signal_chunked_status(csm_ctx* ctx, void* workspace);
/*
 * The two together for narrow sweep panels (C3): every look-back Js[q] (1 <= nJ <= 4, host
 * arrays as csm_momentum_multi) from ONE time-chunked scan -- one summary / fold for max(J) (plus
 * each J's subset-ffilled price) and one chunked multi-J scan instead of three launches per J.
 * Each (M[q], NR[q], ids[q]) equals csm_momentum(PM, Js[q], skip) (+ its ids) bit for bit.  ids
 * nullable (else a host array of device uint16 [T_m][N]).  max(J) + skip <= 16, even N, 16-B
 * aligned PM / M / NR / workspace.  workspace: csm_momentum_multi_chunked_workspace(T_m, N,
 * max(J), skip, C) bytes.
 */
int64_t csm_momentum_multi_chunked_workspace(int32_t T_m, int64_t N, int32_t Jmax, int32_t skip,
                                             int32_t C);
int csm_momentum_multi_chunked(csm_ctx* ctx, const double* PM, int32_t T_m, int64_t N,
                               const int32_t* Js, int32_t nJ, int32_t skip, int32_t C,
                               double* const* M, double* const* NR, uint16_t* const* ids,
                               void* workspace);

/*
 * Fused month-end aggregation + scan in one pass over the daily panel (csm_month_end then
 * csm_momentum without the PM round trip).  Same outputs and carry contract as
 * csm_momentum; PM and R nullable; no volume.  max_month_days (HOST value: the longest
 * month in days) must be <= 32.  Even N with 16-B aligned P takes 16-B row loads.
 */
int csm_signal(csm_ctx* ctx, const double* P, int64_t T_d, int64_t N, const int64_t* month_start,
               int32_t T_m, int32_t max_month_days, int32_t J, int32_t skip, double* PM,
               double* R, double* M, double* NR, const double* carry, const double* next_pm,
               double* carry_out);

/*
 * csm_signal (no carry) that also writes ids[T_m][N] (uint16, 8-B aligned, N % 4 == 0): each
 * mom_J's bucket under the fixed monotone map of csm_deciles_ids (0xFFFF = NaN), so the decile
 * pass reads 2 B per cell instead of 8.  min_month_days (HOST value: the shortest interior
 * month in days; 0 = unknown) is accepted for ABI stability and not used by this build.
 */
int csm_signal_ids(csm_ctx* ctx, const double* P, int64_t T_d, int64_t N,
                   const int64_t* month_start, int32_t T_m, int32_t max_month_days,
                   int32_t min_month_days, int32_t J, int32_t skip, double* PM, double* R,
                   double* M, double* NR, uint16_t* ids);

/*
 * Per-date qcut labels, fused with the equal-weight decile means.  Replaces
 * run_demo.py:18-29 (assign_deciles_per_date via pd.qcut(duplicates='drop')),
 * run_demo.py:46 (groupby('date').transform) and run_demo.py:49-55 (dropna +
 * groupby(['date','decile']).next_ret.mean()).
 *   M[T_m][N]     signal (NaN = not ranked)
 *   NR[T_m][N]    nullable: next-row returns; when NULL, EW/CNT are not produced
 *   qtable        HOST pointer, n_bins+1 quantile levels as NumPy's percentile sees them
 *                 ((linspace(0,1,n+1)*100)/100)
 *   L[T_m][N]     out int8 labels, -1 = NaN
 *   EW[T_m][n_bins]  out, nullable: mean next_ret per (date, label), NaN if empty
 *   CNT[T_m][n_bins] out, nullable: row counts per (date, label)
 *   NV[T_m]       out, nullable: ranked rows per date
 * n_bins in {2,3,4,5,10,20} (any n_bins in [1,20] when NR == NULL).
 */
int csm_deciles(csm_ctx* ctx, const double* M, const double* NR, int32_t T_m, int64_t N,
                int32_t n_bins, const double* qtable, int8_t* L, double* EW, int32_t* CNT,
                int32_t* NV);

/*
 * csm_deciles with the ids of csm_signal_ids: the same labels / EW / CNT / NV bit for bit;
 * M is read only for the cells whose bucket holds an order statistic, an interior edge, or
 * the row's min / max.  N % 4 == 0, 16-B aligned M / NR, 4-B aligned L.
 */
int csm_deciles_ids(csm_ctx* ctx, const double* M, const double* NR, const uint16_t* ids,
                    int32_t T_m, int64_t N, int32_t n_bins, const double* qtable, int8_t* L,
                    double* EW, int32_t* CNT, int32_t* NV);

/*
 * csm_deciles_ids + csm_long_short in one call (run_demo.py:46-67).  Narrow rows (N <= 16384,
 * C2): one launch, the decile pass's last workgroup forms LS[T_m] from every date's EW / CNT
 * (the context's arrival counter; concurrent calls of one context on two streams are not
 * supported).  Wider rows: the long-short kernel follows the decile pass.  NR, EW, CNT and LS
 * are required; the same labels / EW / CNT / NV / LS bits as the two calls.
 */
int csm_deciles_ids_ls(csm_ctx* ctx, const double* M, const double* NR, const uint16_t* ids,
                       int32_t T_m, int64_t N, int32_t n_bins, const double* qtable, int8_t* L,
                       double* EW, int32_t* CNT, int32_t* NV, double* LS);

/*
 * csm_deciles_ids without decile sums, for legs-only accounting (csm_cohort_sums_legs /
 * csm_portfolio_from_cohorts_legs, sweep.SweepConfig.legs_only): with n_bins >= 4 the labels
 * 0 and n_bins - 1 and the NaN label (-1) are exactly csm_deciles_ids's, every other ranked
 * cell gets SOME label in [1, n_bins - 2] (the interior edges' order statistics are not
 * selected).  n_bins < 4: exactly csm_deciles_ids.  NV as there (nullable).
 */
int csm_deciles_ids_legs(csm_ctx* ctx, const double* M, const uint16_t* ids, int32_t T_m,
                         int64_t N, int32_t n_bins, const double* qtable, int8_t* L, int32_t* NV);

/*
 * The whole K = 1 path of run_demo.py:31-67 in one call: fused month-end + scan (csm_signal,
 * with ids when N % 4 == 0 and the row is wide), per-date labels fused with the decile means
 * (csm_deciles / csm_deciles_ids), long-short (csm_long_short).  Arguments as in those calls
 * (min_month_days as in csm_signal_ids);
 * PM, R, NV nullable; qtable HOST.  The ids live in a context-owned workspace (T_m * N * 2 B,
 * grown on first use).
 */
int csm_pipeline(csm_ctx* ctx, const double* P, int64_t T_d, int64_t N, const int64_t* month_start,
                 int32_t T_m, int32_t max_month_days, int32_t min_month_days, int32_t J,
                 int32_t skip, int32_t n_bins,
                 const double* qtable, double* PM, double* R, double* M, double* NR, int8_t* L,
                 double* EW, int32_t* CNT, int32_t* NV, double* LS);

/*
 * Long-short series.  Replaces run_demo.py:57-67: top minus bottom label mean when both
 * columns occur anywhere in the panel, else per-date max minus min; NaN = dropped date.
 *   EW, CNT [T_m][n_bins] from csm_deciles;  LS[T_m] out.
 */
int csm_long_short(csm_ctx* ctx, const double* EW, const int32_t* CNT, int32_t T_m,
                   int32_t n_bins, double* LS);

/*
 * Date-shard summary of a shard's month prices (prefix-independent), [S][N] float64 with
 * S = 6 + J + skip + 1 (layout in DESIGN.md / oracle shard_summary).  No reference
 * counterpart: it is the exchange record of the multi-GPU date sharding.
 */
int csm_shard_summary(csm_ctx* ctx, const double* PM, int32_t T_m, int64_t N, int32_t J,
                      int32_t skip, double* out);

/*
 * Fold the all-gathered summaries [G][S][N] into shard g's inherited scan state
 * (carry [(J+skip)+2][N]) and next_pm[N], bit-exactly equal to an unsharded scan.
 */
int csm_fold_carry(csm_ctx* ctx, const double* summaries, int32_t G, int32_t g, int64_t N,
                   int32_t J, int32_t skip, double* carry, double* next_pm);

/*
 * Speculative date shards (the fused multi-GPU pass; no reference counterpart).
 * csm_signal_shard: csm_signal over this rank's months from an EMPTY scan state, before the
 *   earlier shards' carry is known (no carry / next_pm).  PM [T_m][N] is required but only its
 *   first and last J + skip + 8 months are written (the calls below re-derive other months
 *   from P where an asset needs them); state [5][N] out: present months, pending ranked row
 *   (-1 none), its subset-ffilled price, first and last present month (-1 none).  T_m >= 1.
 * csm_shard_summary_state: the csm_shard_summary record of the shard's month prices, bit for
 *   bit, from short walks at both ends of each asset's present months.
 * csm_shard_repair: with carry / next_pm from csm_fold_carry, rewrites R (nullable) / M / NR
 *   where the true carry changes them and finishes the pending rows, so the result equals
 *   csm_momentum(month prices, carry, next_pm) bit for bit.  J + skip <= 128.
 * P / month_start / PM / state are the csm_signal_shard call's.
 */
int csm_signal_shard(csm_ctx* ctx, const double* P, int64_t T_d, int64_t N,
                     const int64_t* month_start, int32_t T_m, int32_t max_month_days, int32_t J,
                     int32_t skip, double* PM, double* R, double* M, double* NR, double* state);
int csm_shard_summary_state(csm_ctx* ctx, const double* P, const int64_t* month_start,
                            const double* PM, int32_t T_m, int64_t N, int32_t J, int32_t skip,
                            const double* state, double* out);
int csm_shard_repair(csm_ctx* ctx, const double* P, const int64_t* month_start, const double* PM,
                     int32_t T_m, int64_t N, int32_t J, int32_t skip, const double* carry,
                     const double* next_pm, const double* state, double* R, double* M,
                     double* NR);
/*
 * The speculative shard pass with bucket ids (for csm_deciles_ids): csm_signal_shard that also
 * writes ids[T_m][N] like csm_signal_ids (N % 4 == 0, 8-B aligned), and csm_shard_repair that
 * rewrites the id of every cell it rewrites.  Same M / NR / R bits as the plain calls.
 */
int csm_signal_shard_ids(csm_ctx* ctx, const double* P, int64_t T_d, int64_t N,
                         const int64_t* month_start, int32_t T_m, int32_t max_month_days,
                         int32_t J, int32_t skip, double* PM, double* R, double* M, double* NR,
                         double* state, uint16_t* ids);
int csm_shard_repair_ids(csm_ctx* ctx, const double* P, const int64_t* month_start,
                         const double* PM, int32_t T_m, int64_t N, int32_t J, int32_t skip,
                         const double* carry, const double* next_pm, const double* state,
                         double* R, double* M, double* NR, uint16_t* ids);

/*
 * Halo date shards (the default multi-GPU pass; no reference counterpart, SURVEY 8(e) and
 * north_star's "J + skip lookback halo").  A rank holds the daily rows of H calendar months
 * before its shard, its T_m shard months and F (0..8) months after it, month_start[H + T_m + F
 * + 1] (day offsets into P, the 'ME' groups of features.py:38).
 * csm_shard_halo: the scan state the halo months leave from an empty state (carry
 *   [(J+skip)+2][N], csm_signal's layout), next_pm[N] = the price of the first forward month
 *   with a row (ABSENT if none), and flags[N]: bit 0 the carry may differ from the one the
 *   whole history leaves (before != 0 -- the panel has months before the halo -- and the halo
 *   lacks two valid prices J + skip present months apart), bit 1 next_pm may differ (after !=
 *   0 -- the panel has months after the forward months -- and no forward row).  halo_pm:
 *   workspace [H + F][N] (the halo and forward months' prices).
 * csm_signal_shard_halo: csm_signal_shard from that carry and next_pm (month_start = the
 *   shard's T_m + 1 offsets, still into P); unflagged assets' outputs are final.
 * csm_shard_need: this rank's exchange bits mask[4][ceil(N / 64)] (bit a % 64 of word a / 64):
 *   row 0 flag bit 0 and a present month in the shard, row 1 flag bit 1 and a pending ranked
 *   row at its end, row 2 a present month, row 3 a present month before the shard's last H
 *   months (the part outside the next rank's halo).
 * csm_shard_union: from every rank's rows [G][4][ceil(N / 64)], the assets some rank needs --
 *   an uncertain carry and a row before that rank's halo, or an uncertain forward price and a
 *   row in a later shard -- as the ascending list idx[min(*count, cap)]; *count its full
 *   length (> cap: overflow -- take the all-gather path).  Same list on every rank.
 * csm_shard_summary_cols: csm_shard_summary_state's record for the listed assets only,
 *   out[S][cap] (columns past *count: an asset with no present month).  All-gather it, fold it
 *   with csm_fold_carry (N = cap), and:
 * csm_shard_repair_cols: csm_shard_repair of the listed assets, their carry / next_pm columns
 *   from that fold ([.][cap]); fcarry = this rank's halo carry (the state the pass started from).
 * csm_shard_fix_cols: the fold and the repair of the listed columns in ONE launch (the halo
 *   pass's default): records = the all-gathered [G][S][cap] records, g = this rank; each listed
 *   column's true carry and forward price are folded from them and every month of the column
 *   is replayed from that carry (the sequential scan: the unsharded pass's R / M / NR / ids).
 */
int csm_shard_halo(csm_ctx* ctx, const double* P, int64_t T_d, int64_t N,
                   const int64_t* month_start, int32_t H, int32_t T_m, int32_t F,
                   int32_t before, int32_t after, int32_t J, int32_t skip, double* halo_pm,
                   double* carry, double* next_pm, uint8_t* flags);
/*
 * csm_signal_halo: csm_shard_halo + csm_signal_shard_halo in ONE launch (the wide shard kernel:
 * even N >= 92160, months of <= 23 day rows; else CSM_E_INVAL -- take the two calls): P and
 * month_start [H + T_m + F + 1] as csm_shard_halo's; the halo state, the forward price and
 * flags [N] (csm_shard_halo's) come from the kernel's prologue, the shard's PM / R / M / NR /
 * state / ids are csm_signal_shard_halo's, bit for bit.
 */
int csm_signal_halo(csm_ctx* ctx, const double* P, int64_t T_d, int64_t N,
                    const int64_t* month_start, int32_t H, int32_t T_m, int32_t F, int32_t before,
                    int32_t after, int32_t max_month_days, int32_t J, int32_t skip, double* PM,
                    double* R, double* M, double* NR, double* state, uint16_t* ids,
                    uint8_t* flags);
int csm_signal_shard_halo(csm_ctx* ctx, const double* P, int64_t T_d, int64_t N,
                          const int64_t* month_start, int32_t T_m, int32_t max_month_days,
                          int32_t J, int32_t skip, const double* carry, const double* next_pm,
                          double* PM, double* R, double* M, double* NR, double* state,
                          uint16_t* ids);
int csm_shard_need(csm_ctx* ctx, const uint8_t* flags, const double* state, int64_t N,
                   int32_t T_m, int32_t H, uint64_t* mask);
int csm_shard_union(csm_ctx* ctx, const uint64_t* masks, int32_t G, int64_t N, int64_t cap,
                    int32_t* idx, int32_t* count);
int csm_shard_summary_cols(csm_ctx* ctx, const double* P, const int64_t* month_start,
                           const double* PM, int32_t T_m, int64_t N, int32_t J, int32_t skip,
                           const double* state, const int32_t* idx, const int32_t* count,
                           int64_t cap, double* out);
int csm_shard_repair_cols(csm_ctx* ctx, const double* P, const int64_t* month_start,
                          const double* PM, int32_t T_m, int64_t N, int32_t J, int32_t skip,
                          const double* carry, const double* next_pm, const double* fcarry,
                          const double* state, const int32_t* idx, const int32_t* count,
                          int64_t cap, double* R, double* M, double* NR, uint16_t* ids);
int csm_shard_fix_cols(csm_ctx* ctx, const double* P, const int64_t* month_start,
                       const double* PM, int32_t T_m, int64_t N, int32_t J, int32_t skip,
                       const double* records, int32_t G, int32_t g, const int32_t* idx,
                       const int32_t* count, int64_t cap, double* R, double* M, double* NR,
                       uint16_t* ids);

/*
 * Portfolio accounting beyond the reference's K = 1 equal-weight case (SURVEY 8(f) rank 2;
 * rules E1..E5 in DESIGN.md section 8 / oracle/portfolio_oracle.py).  The reference counterpart
 * is run_demo.py:49-67 (K = 1, equal weight, no costs), which this collapses to.
 * Panels are batched [T_m][B][N] (B cross-sections per month row; B = 1 for one panel).
 *   L         int8 labels from csm_deciles (-1 = not ranked)
 *   NR        next-row returns (the return held over (t, t+1])
 *   W         nullable: formation weights (value weighting, e.g. market cap); NULL = equal
 *   K         holding months: month t averages the cohorts formed at t-K+1 .. t
 *   half_spread, k_impact, aum, ADV (nullable [T_m][B][N] dollar ADV), SIG (nullable
 *             volatility, NaN/NULL -> 0.02): the cost model of src/execution_models.py:4-12
 *   PR [T_m][B][n_bins]  overlapped decile returns;  LS [T_m][B] long-short (NaN = dropped)
 *   TURN, COST, NET [T_m][B] nullable: long-short turnover (1/2 sum |dw|), cost, LS - COST
 *   workspace: device buffer of csm_portfolio_workspace(T_m, B, N, n_bins, K) bytes
 * n_bins in {2,3,4,5,10,20,30}.
 */
int64_t csm_portfolio_workspace(int32_t T_m, int32_t B, int64_t N, int32_t n_bins, int32_t K);
int csm_portfolio(csm_ctx* ctx, const int8_t* L, const double* NR, const double* W, int32_t T_m,
                  int32_t B, int64_t N, int32_t n_bins, int32_t K, double half_spread,
                  double k_impact, double aum, const double* ADV, const double* SIG, double* PR,
                  double* LS, double* TURN, double* COST, double* NET, void* workspace);

/*
 * The two halves of csm_portfolio, for sweeps over K: cohort sums do not depend on the
 * holding period, so one csm_cohort_sums pass with Kmax cohorts (workspace of
 * csm_portfolio_workspace(T_m, B, N, n_bins, Kmax) bytes) serves csm_portfolio_from_cohorts
 * for every K <= Kmax (same L / W; outputs as csm_portfolio).
 */
int csm_cohort_sums(csm_ctx* ctx, const int8_t* L, const double* NR, const double* W, int32_t T_m,
                    int32_t B, int64_t N, int32_t n_bins, int32_t Kmax, void* workspace);
int csm_portfolio_from_cohorts(csm_ctx* ctx, const int8_t* L, const double* W, int32_t T_m,
                               int32_t B, int64_t N, int32_t n_bins, int32_t Kmax, int32_t K,
                               double half_spread, double k_impact, double aum, const double* ADV,
                               const double* SIG, double* PR, double* LS, double* TURN,
                               double* COST, double* NET, void* workspace);
/* Several holding periods at once (Ks: HOST array of nK values <= Kmax): outputs stacked
 * over K -- PR [nK][T_m][B][n_bins], LS / TURN / COST / NET [nK][T_m][B]; the turnover pass
 * loads each cell's labels once for up to 4 K values. */
int csm_portfolio_from_cohorts_multi(csm_ctx* ctx, const int8_t* L, const double* W,
                                     int32_t T_m, int32_t B, int64_t N, int32_t n_bins,
                                     int32_t Kmax, int32_t nK, const int32_t* Ks,
                                     double half_spread, double k_impact, double aum,
                                     const double* ADV, const double* SIG, double* PR, double* LS,
                                     double* TURN, double* COST, double* NET, void* workspace);

/*
 * Legs-only accounting for sweeps whose outputs are the long-short statistics (SweepRunner:
 * LS / TURN / COST / NET per strategy): csm_cohort_sums_legs sorts and sums only the two legs
 * (deciles 0 and n_bins - 1; rows of <= 7168 assets), csm_portfolio_from_cohorts_legs takes the
 * multi-K accounting from them -- LS, TURN, COST and NET equal the full path's bit for bit, PR
 * holds the two legs (NaN elsewhere).  The reference's long-short rule needs every decile only
 * when a panel lacks one leg's column (run_demo.py:60-65): then *need_full (device int32, set to
 * 0 by the caller) becomes 1 and the caller reruns the full csm_cohort_sums /
 * csm_portfolio_from_cohorts_multi.  The legs pass stores its partials in a two-leg layout and
 * records the layout in the workspace (the accounting reads it there): a full
 * csm_portfolio_from_cohorts* needs the full cohort sums, as before.
 */
/*
 * Equal-weight cohort sums of nJ (<= 4) label panels L[q] that share one next_ret panel NR (the
 * bootstrap sweep's shared next_ret, csm_boot_scan): each workspace[q] (csm_portfolio_workspace
 * bytes) ends up as csm_cohort_sums(_legs)(L[q], NR, NULL, ..., workspace[q]) leaves it, bit for
 * bit, but each month's return row is read once for every J (one launch) where the segment path
 * applies.  legs: 1 = csm_cohort_sums_legs.  Then csm_portfolio_from_cohorts_* per J.
 */
int csm_cohort_sums_js(csm_ctx* ctx, int32_t nJ, const int8_t* const* L, const double* NR,
                       int32_t T_m, int32_t B, int64_t N, int32_t n_bins, int32_t Kmax,
                       int32_t legs, void* const* workspaces);
int csm_cohort_sums_legs(csm_ctx* ctx, const int8_t* L, const double* NR, const double* W,
                         int32_t T_m, int32_t B, int64_t N, int32_t n_bins, int32_t Kmax,
                         void* workspace);
int csm_portfolio_from_cohorts_legs(csm_ctx* ctx, const int8_t* L, const double* W,
                                    int32_t T_m, int32_t B, int64_t N, int32_t n_bins,
                                    int32_t Kmax, int32_t nK, const int32_t* Ks,
                                    double half_spread, double k_impact, double aum,
                                    const double* ADV, const double* SIG, double* PR, double* LS,
                                    double* TURN, double* COST, double* NET, void* workspace,
                                    int32_t* need_full);

/*
 * The cohort sums and accounting of B = G * Bg panels whose labels / next_ret are stored
 * group-major -- L, NR [G][T_m][Bg][N]: G blocks, e.g. G look-backs' label panels as one decile
 * pass over the stacked rows writes them -- and whose weights / ADV / vol are shared by the G
 * groups -- W, ADV, SIG [T_m][Bg][N] (nullable as above).  Each call equals its plain-layout
 * counterpart (csm_cohort_sums(_legs), csm_portfolio_from_cohorts_multi / _legs) on the
 * side-by-side panels ([T_m][G * Bg][N], panel g * Bg + p = group g's panel p, weights repeated
 * per group) bit for bit, outputs and workspace included (csm_portfolio_workspace(T_m, G * Bg,
 * N, n_bins, Kmax) bytes; outputs [nK][T_m][G * Bg]), without those copies.  legs: 1 = the
 * legs-only forms (rows of <= 7168 assets; need_full as csm_portfolio_from_cohorts_legs).
 */
int csm_cohort_sums_grouped(csm_ctx* ctx, int32_t G, const int8_t* L, const double* NR,
                            const double* W, int32_t T_m, int32_t Bg, int64_t N, int32_t n_bins,
                            int32_t Kmax, int32_t legs, void* workspace);

/*
 * csm_cohort_sums_js for label panels stored group-major, L int8 [nJ][T_m][B * N] (the look-backs'
 * panels as one stacked decile pass writes them), into ONE workspace laid out for nJ * B panels
 * (csm_portfolio_workspace(T_m, nJ * B, ...); J q's panel b is panel q * B + b, as
 * csm_cohort_sums_grouped lays it out): one label-sort launch for every J and each month's
 * return row staged once for every J.  csm_portfolio_from_cohorts_grouped(G = nJ, Bg = B) then
 * accounts every J in one launch set.  Where csm_portfolio_plan(T_m, B, ...) equals
 * csm_portfolio_plan(T_m, nJ * B, ...), every J's results are csm_cohort_sums_js's bit for bit.
 */
int csm_cohort_sums_js_grouped(csm_ctx* ctx, int32_t nJ, const int8_t* L, const double* NR,
                               int32_t T_m, int32_t B, int64_t N, int32_t n_bins, int32_t Kmax,
                               int32_t legs, void* workspace);

/*
 * The chunk plan of a portfolio call on (T_m, B, N, n_bins, K): cohort chunks C in the low 32
 * bits, turnover chunks Ct in the high ones (-1 on bad arguments).  Two calls with the same plan
 * give each panel the same partial sums, so their per-panel results are the same bits.
 */
int64_t csm_portfolio_plan(int32_t T_m, int32_t B, int64_t N, int32_t n_bins, int32_t K);
int csm_portfolio_from_cohorts_grouped(csm_ctx* ctx, int32_t G, const int8_t* L, const double* W,
                                       int32_t T_m, int32_t Bg, int64_t N, int32_t n_bins,
                                       int32_t Kmax, int32_t nK, const int32_t* Ks,
                                       double half_spread, double k_impact, double aum,
                                       const double* ADV, const double* SIG, double* PR,
                                       double* LS, double* TURN, double* COST, double* NET,
                                       void* workspace, int32_t legs, int32_t* need_full);

/*
 * Performance summary per (strategy, panel) of stacked long-short series (LS, and the
 * nullable-together TURN / COST / NET, each [nS][T_m][B]): out [nS][B][7] = months, mean,
 * Sharpe (src/utils.py:8-16 at `freq` periods a year, ddof = 1), mean turnover, mean cost,
 * net mean, net Sharpe; NaN months dropped (run_demo.py:67).
 */
int csm_summary(csm_ctx* ctx, const double* LS, const double* TURN, const double* COST,
                const double* NET, int32_t nS, int32_t T_m, int32_t B, double freq,
                double* out);

/*
 * Stationary month bootstrap (BASELINE config C5; rule E6): panels b0 .. b0+B-1 of the base
 * month-return panel R[T_m][N] (csm_momentum's R; NaN = no row).  src[B][T_m] int32 out: the
 * source months; PMb[T_m][B][N] out: month prices p0 * prod(1 + r) over the resampled months,
 * ABSENT where the source return is NaN.  The random stream is splitmix64 keyed by
 * (seed, panel, month), so panel b is the same on every device and shard.
 */
int csm_bootstrap(csm_ctx* ctx, const double* R, int32_t T_m, int64_t N, int32_t B, int64_t b0,
                  uint64_t seed, double mean_block, double p0, int32_t* src, double* PMb);

/*
 * csm_bootstrap fused into csm_momentum_multi_ids for the bootstrap sweep (C5): the resampled
 * prices are generated in registers from R (csm_bootstrap's arithmetic, never written), scanned
 * for every J of Js in one pass, and written as M[nJ] (+ IDS[nJ], nullable) equal bit for bit to
 * csm_momentum_multi_ids on csm_bootstrap's panel, plus ONE next_ret panel NR [T_m][B][N] shared
 * by every J: equal to each J's next_ret on every row that J ranks (all the portfolio reads).
 *   src [B][T_m] out (as csm_bootstrap);  M[q] / IDS[q] / NR [T_m][B][N] out;
 *   bad: device int32, set to 1 when a generated price is not finite and non-zero (the shared
 *   next_ret is then not exact: rerun the batch on the csm_bootstrap path).
 * N even, 1 <= nJ <= 4, J + skip <= 16, 16-B aligned R / M / NR, 4-B aligned ids.
 */
int csm_boot_scan(csm_ctx* ctx, const double* R, int32_t T_m, int64_t N, int32_t B, int64_t b0,
                  uint64_t seed, double mean_block, double p0, const int32_t* Js, int32_t nJ,
                  int32_t skip, int32_t* src, double* const* M, uint16_t* const* IDS, double* NR,
                  int32_t* bad);

/*
 * Share-turnover features, replacing src/features.py:60-107 (compute_monthly_turnover) on the
 * dense monthly layout (rule T1): per present row adv = VOL / 21, shares = so[a] when not NaN
 * else trunc(mcap[a] / PM) when mcap != 0 and PM > 0 (NaN when that is not finite),
 * turnover = adv / shares when shares > 0, and turn_avg = pandas' rolling(lookback,
 * min_periods=1).mean() over the asset's present rows (bit-exact restatement).
 *   PM, VOL [T_m][N] from csm_month_end;  so, mcap [N] (NaN = not given)
 *   ADV, SH, TURN, TAVG [T_m][N] out (NaN where the asset has no row); lookback in [1, 48]
 */
int csm_turnover_features(csm_ctx* ctx, const double* PM, const double* VOL, const double* so,
                          const double* mcap, int32_t T_m, int64_t N, int32_t lookback,
                          double* ADV, double* SH, double* TURN, double* TAVG);

/*
 * Momentum x volume double sort helpers (LeSw00 section II; rule T2):
 *   Xm = X where M is valid, NaN elsewhere (the tercile universe; nullable)
 *   Lc = n_vol * Lm + Lv where both labels are valid, -1 elsewhere (nullable)
 * The cell returns then come from csm_portfolio with n_bins = n_mom * n_vol (30 supported).
 */
int csm_double_sort_labels(csm_ctx* ctx, const double* M, const double* X, const int8_t* Lm,
                           const int8_t* Lv, int32_t T_m, int64_t N, int32_t n_vol, double* Xm,
                           int8_t* Lc);

/*
 * The date-shard collectives over RCCL (xGMI on one node), for hosts that shard
 * run_demo.py:31-67 without torch.distributed: csm_comm_unique_id fills CSM_UNIQUE_ID_BYTES
 * (host memory) on ONE rank; the bytes reach the other ranks out of band; every rank calls
 * csm_allgather_init with them (one communicator per context, on the context's device); then
 * csm_allgather gathers `bytes` from every rank into recv (device, nranks * bytes, rank order)
 * on the context's stream -- collective 1 (the [S][N] shard summaries for csm_fold_carry) and
 * collective 2 (the per-date decile means / counts for csm_long_short).  csm_allgather_free
 * (also done by csm_destroy) releases the communicator.  RCCL is loaded at first use;
 * CSM_E_RCCL when it is missing or a call fails.
 */
int csm_comm_unique_id(void* unique_id);
int csm_allgather_init(csm_ctx* ctx, const void* unique_id, int32_t rank, int32_t nranks);
int csm_allgather(csm_ctx* ctx, const void* send, void* recv, int64_t bytes);
int csm_allgather_free(csm_ctx* ctx);

#ifdef __cplusplus
}
#endif

#endif /* CSMOM_H */
