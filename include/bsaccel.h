/*
 * bsaccel.h -- C ABI of the MI355X-native BlueSky CD / MVP / kinematics path.
 *
 * One shared library (bluesky_amd/libbsaccel.so, HIP for gfx950) that the
 * Python drop-ins in bluesky_amd/ bind through ctypes.  Plain pointers and
 * sizes only; no exceptions cross the ABI.  Every entry point returns an int
 * status: 0 = OK, < 0 = error (message via bsa_last_error(ctx)).
 *
 * Reference interfaces replaced (paths relative to the BlueSky checkout):
 *   bsa_detect / bsa_fetch_pairs
 *       bluesky/traffic/asas/StateBasedCD.py:7-103   detect(ownship, intruder, RPZ, HPZ, tlookahead)
 *       bluesky/tools/geo.py:110-162                 qdrdist_matrix (fused, never materialised)
 *       bluesky/traffic/asas/src_cpp/casas.cpp:12-106 casas.detect (native variant it supersedes)
 *   bsa_mvp
 *       bluesky/traffic/asas/MVP.py:14-300           resolve / MVP / prioRules
 *   bsa_kinematics
 *       bluesky/traffic/traffic.py:425-483           UpdateAirSpeed / UpdateGroundSpeed / UpdatePosition
 *       bluesky/tools/aero.py:62-147                 vatmos / vtas2cas / vtas2mach (inlined)
 *   bsa_set_windfield (winddim 2)
 *       bluesky/traffic/windfield.py:158-179         Windfield.getdata, 2-D field
 *   bsa_qdrdist
 *       bluesky/tools/geo.py:110-162,347-363         qdrdist_matrix / kwikqdrdist_matrix, materialised
 *   bsa_sim_set_limits
 *       bluesky/traffic/pilot.py:65-68 + performance/openap/perfoap.py:185-209  applylimits (OpenAP)
 *   bsa_sim_acdata_*
 *       bluesky/simulation/qtgl/screenio.py:194-239  send_aircraft_data (ACDATA stream fields)
 *   bsa_sim_*     GPU-resident chain of the above, no reference equivalent
 *   bsa_comm_*    RCCL row-sharded multi-GPU mode, no reference equivalent
 *
 * Threading: a context is bound to one HIP device and one stream and is not
 * thread-safe; use one context per host thread (the BlueSky sim loop is
 * single-threaded, bluesky/network/detached.py:34-41).
 */
#ifndef BSACCEL_H
#define BSACCEL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BSA_ABI_VERSION 1

typedef struct bsa_ctx bsa_ctx;

/* detect flags */
#define BSA_FLAG_WITH_DCPA 1 /* also produce dcpa = sqrt(max(dcpa2,0)) per conflict */
#define BSA_FLAG_NOPRUNE   2 /* test aid: treat every pair as a candidate (disables the exact-safe prefilter) */
#define BSA_FLAG_RESORT    4 /* recompute the spatial order now (it is otherwise reused for up to
                                8 calls; results never depend on it, only the speed does) */
#define BSA_FLAG_KWIK      8 /* opt-in flat-earth variant: geo.kwikqdrdist_matrix
                                (geo.py:347-363) replaces qdrdist_matrix in StateBasedCD.detect, its
                                metre distance passed on in nm; qdr in [0, 360) */
#define BSA_FLAG_STAGE1_T0 16 /* test aid: prefilter stage 1 at the t = 0 positions with the full
                                look-ahead reach instead of the look-ahead midpoints (DESIGN.md
                                3.2b); results are identical, only the culling differs */

/* ---------------------------------------------------------------- lifecycle */

/* ABI version of the loaded library (== BSA_ABI_VERSION it was built with). */
int bsa_abi_version(void);

/* Number of visible HIP devices (>= 0), or < 0 on runtime error. */
int bsa_device_count(void);

/* Create a context on HIP device `device`.  Returns NULL on failure; the
 * reason is then available from bsa_last_error(NULL). */
bsa_ctx *bsa_create(int device);
void bsa_destroy(bsa_ctx *ctx);

/* Last error message of `ctx` (or of the failed bsa_create when ctx==NULL).
 * The string is owned by the library and valid until the next call. */
const char *bsa_last_error(const bsa_ctx *ctx);

/* Block until all work queued on the context's stream has finished. */
int bsa_sync(bsa_ctx *ctx);

/* ---------------------------------------------------------------- state
 * Replaces reading bs.traf.{lat,lon,trk,gs,alt,vs} inside StateBasedCD.detect
 * (StateBasedCD.py:16-17,30-37,65-69).  Host arrays are C-contiguous float64
 * of length n, borrowed for the duration of the call (copied to HBM).
 * Units as in bluesky Traffic: lat/lon/trk [deg], gs [m/s], alt [m], vs [m/s]. */
int bsa_set_state(bsa_ctx *ctx, int64_t n,
                  const double *lat, const double *lon, const double *trk,
                  const double *gs, const double *alt, const double *vs);

/* Optional distinct intruder set (detect(ownship, intruder, ...) with
 * intruder is not ownship).  n must equal the ownship n; n == 0 clears it
 * (intruder = ownship again).  Must be called after bsa_set_state. */
int bsa_set_intruder(bsa_ctx *ctx, int64_t n,
                     const double *lat, const double *lon, const double *trk,
                     const double *gs, const double *alt, const double *vs);

/* ---------------------------------------------------------------- detect
 * StateBasedCD.detect for ownship rows [row_begin, row_end) against all n
 * intruder columns (row_end <= 0 means n).  rpz/hpz in metres, tla in
 * seconds.  On success *n_conf / *n_los hold the number of conflict and
 * loss-of-separation pairs of these rows; the pairs stay on the device until
 * the next bsa_detect (bsa_mvp consumes them). */
int bsa_detect(bsa_ctx *ctx, double rpz, double hpz, double tla, int flags,
               int64_t row_begin, int64_t row_end,
               int64_t *n_conf, int64_t *n_los);

/* Copy the last detect's results to caller-allocated host arrays, in the
 * reference's row-major (i, j) order (StateBasedCD.py:93-101):
 *   ci, cj, qdr[deg], dist[m], tcpa[s], tinconf[s]       n_conf entries each
 *   dcpa[m] (n_conf, may be NULL; needs BSA_FLAG_WITH_DCPA)
 *   li, lj                                                n_los entries each
 *   inconf (uint8 0/1), tcpamax[s]                        row_end-row_begin entries
 * Any pointer may be NULL to skip that output.  Non-finite inputs follow the
 * reference (StateBasedCD.py:90): tcpamax is NaN on every row when some
 * column's position / velocity is not finite, and on one row when only that
 * row's is; the pairs are the finite aircraft's. */
int bsa_fetch_pairs(bsa_ctx *ctx,
                    int32_t *ci, int32_t *cj, double *qdr, double *dist,
                    double *tcpa, double *tinconf, double *dcpa,
                    int32_t *li, int32_t *lj,
                    uint8_t *inconf, double *tcpamax);

/* Candidate-pair count of the last detect (pairs that passed the
 * conservative prefilter and were evaluated exactly in fp64). */
int bsa_last_candidates(bsa_ctx *ctx, int64_t *n_candidates);

/* Candidate-list capacity (pairs surviving the prefilter) for the next
 * detects; rounded up to a multiple of the shard count.  Detects grow it on
 * overflow (with a retry), so this is a tuning / testing knob only.  Once the
 * resident sim's ASAS bookkeeping has started it also sets the resopairs
 * capacity (grown the same way). */
int bsa_set_candidate_capacity(bsa_ctx *ctx, int64_t capacity);

/* K2 (canonical order) row buckets: width w (1..64) pairs per row are
 * placed by K1b directly, K2 ranks each pair inside its row's bucket; a row
 * with more pairs makes the detect retry with a wider bucket (beyond 64: the
 * scatter into row segments, width 0).  Default 8.  Results never depend on
 * it (tests set it to exercise every path). */
int bsa_set_row_bucket(bsa_ctx *ctx, int width);
/* K1b (the exact fp64 evaluation of the prefilter's candidates) fused into
 * the prefilter's launch (on by default; stored records, row buckets, not
 * KWIK / candidate reuse): each prefilter workgroup evaluates the candidates
 * it produced at the end of its sweep.  max_records (0..64, default 64): the
 * mid-sweep flushes a wave records for that; a wave that flushes more makes
 * the detect retry with K1b as its own launch (0 forces that retry whenever
 * a wave flushes mid-sweep: a testing knob).  Results never depend on it. */
int bsa_set_exact_fusion(bsa_ctx *ctx, int on, int max_records);
/* [0] detects enqueued with K1b fused, [1] of them retried unfused (a wave ran
 * out of flush records), [2] whether the last detect fused (0 / 1). */
int bsa_exact_fusion_stats(bsa_ctx *ctx, int64_t *out3);
/* Candidate-list reuse across detects (own == intruder, whole row range, not
 * KWIK / NOPRUNE).  A detect that builds the list inflates
 * every aircraft's reach by a horizontal budget sigma_h [m] and a vertical
 * budget (sigma_v [m] at first, then adapted per aircraft to its own drift
 * rate, up to 4 sigma_v); later detects skip the sweep (K0c/K0d/K1a) and
 * re-evaluate that list exactly, until some aircraft's drift since the build
 * (position, velocity, altitude, vertical speed) exceeds its budget, a
 * re-sort, a parameter change or an overflow -- checked on the device, so the
 * results are identical to a full detect.  Off by default. */
int bsa_set_candidate_reuse(bsa_ctx *ctx, int on, double sigma_h, double sigma_v);
/* List builds and detects since the last bsa_timing_reset. */
int bsa_reuse_stats(bsa_ctx *ctx, int64_t *builds, int64_t *detects);
/* Largest fraction of its horizontal [0] / vertical [1] budget any aircraft
 * had used at the last detect (> 1 triggered a build; 0 after a forced one). */
int bsa_reuse_budget_use(bsa_ctx *ctx, double *use2);
/* Tile-pair list reuse in the resident sim step (on by
 * default): the detect's coarse cull -- which (512-row tile, 512-column tile,
 * 64-row slice) items the prefilter sweeps (K0d) -- is built on boxes grown by
 * sigma_h [m] horizontally (and proportionally in reach) and sigma_v [m]
 * vertically, and kept while every aircraft's prefilter record stays within
 * those distances of its record at the build (K4' checks each record it
 * prepares; the first one outside makes the next detect rebuild on the
 * device).  Every pair is still tested and evaluated at every detect, so the
 * results are identical with it on or off.  off: every detect builds. */
int bsa_set_tile_reuse(bsa_ctx *ctx, int on, double sigma_h, double sigma_v);
/* [0] tile-pair list builds, [1] detects that used the kept or a fresh list,
 * since the sim's first such detect (device counters). */
int bsa_tile_reuse_stats(bsa_ctx *ctx, int64_t *out2);
/* Host-known list decisions in the resident step (HK): on =
 * 0 lets the device decide every rebuild (the round-5 behaviour, one K0d /
 * halo plan launch per detect); f in (0, 4] is the fraction of the drift
 * budgets past which the device predicts a rebuild two detects ahead (f > 1:
 * predictions come late, kept lists go stale and their steps re-run -- a
 * testing knob).  Results never depend on either. */
int bsa_set_hk(bsa_ctx *ctx, int on, double f);
/* out6 = {host-kept detects, host-built detects, waits for a prediction,
 * stale aborts (re-run steps), device-decided detects after them, on} */
int bsa_hk_stats(bsa_ctx *ctx, int64_t *out6);
/* Halo overlap of the row-sharded resident step: on a detect
 * that keeps its halo plan, the halo send / recv, the received tiles' K0b and
 * the sweep of the halo column tiles run on a second stream while the own
 * tiles' K0b and sweep run; joined before K1b.  mode 0 off (default), 1
 * several ranks, 2 also the one-GPU probe (bsa_sim_probe_rank: its cost with
 * no exchange to hide).  Results never depend on it.  out: overlapped detects. */
int bsa_set_halo_overlap(bsa_ctx *ctx, int mode);
int bsa_halo_overlap_count(bsa_ctx *ctx, int64_t *out1);

/* Tile pairs (512 rows x 512 columns) of the last detect that survived the
 * bounding-box cull, the total number of tile pairs, and the number of
 * (64-row x 8-column) blocks the prefilter actually swept (each block is
 * BSA_PF_BLOCK_PAIRS stage-1 pair tests). */
#define BSA_PF_BLOCK_PAIRS 512
int bsa_last_tiles(bsa_ctx *ctx, int64_t *kept, int64_t *total, int64_t *groups);

/* Device time of the last detect's stages in milliseconds, measured with
 * HIP events on the context stream: [0] spatial order + records + tile cull,
 * [1] prefilter, [2] exact, [3] sort+gather, [4] whole detect. */
int bsa_last_timings(bsa_ctx *ctx, double *ms5);

/* Timing / statistics accumulation over many detects (benchmarking): reset
 * forgets every recorded detect; summary waits for the stream and returns the
 * MEAN stage durations over the detects since the reset (same layout as
 * bsa_last_timings) and the SUMS stats4 = {(64-row x 16-column) prefilter
 * blocks swept, candidates, surviving tile pairs, detects}. */
int bsa_timing_reset(bsa_ctx *ctx);
int bsa_timing_summary(bsa_ctx *ctx, double *ms5, int64_t *stats4);
/* Record the stage events of one detect in `every` (default 1 = all; 0 =
 * none; counted from the last bsa_timing_reset, whose first detect is timed).
 * Each event record costs a ~5 us gap before the next kernel, so the bench
 * samples; bsa_last_timings then reports the last timed detect and
 * bsa_timing_summary averages the timed ones. */
int bsa_set_timing_sample(bsa_ctx *ctx, int every);

/* ---------------------------------------------------------------- MVP
 * MVP.resolve (bluesky/traffic/asas/MVP.py:14-143) on the device-resident
 * conflict pairs of the last bsa_detect (rows [row_begin,row_end) of it).
 * Scalars as held by ASAS (asas.py:81-112): Rm = R*mar, dhm = dh*mar, vmin/
 * vmax/vsmin/vsmax in m/s; switches 0/1; priocode one of BSA_PRIO_* (any
 * other value = a code prioRules does not know: no change). */
#define BSA_PRIO_NONE 0
#define BSA_PRIO_FF1  1
#define BSA_PRIO_FF2  2
#define BSA_PRIO_FF3  3
#define BSA_PRIO_LAY1 4
#define BSA_PRIO_LAY2 5
typedef struct bsa_mvp_params {
  double Rm, dhm, dtlookahead, vmin, vmax, vsmin, vsmax;
  int32_t swresohoriz, swresospd, swresohdg, swresovert;
  int32_t swprio, priocode;
  int32_t swnoreso, swresooff;
} bsa_mvp_params;

/* Load externally detected conflict pairs (e.g. from the numpy StateBasedCD)
 * as if they were the last detect's, for all n rows: P pairs in confpair
 * order with ci non-decreasing (row-major, as detect returns them), and their
 * qdr [deg], dist [m], tcpa [s], tLOS [s] (MVP.py:33). */
int bsa_set_pairs(bsa_ctx *ctx, int64_t P, const int32_t *ci, const int32_t *cj,
                  const double *qdr, const double *dist, const double *tcpa,
                  const double *tlos);

/* Inputs (host, length n = state n): gseast, gsnorth, selalt, apvs (= traf.ap.vs),
 * noreso / resooff: uint8 per aircraft (membership of asas.noresolst /
 * asas.resoofflst; NULL = empty list).  vs/alt/trk/gs come from bsa_set_state.
 * asas_alt: persistent asas.alt of the detect rows, read-modify-write.
 * Outputs (detect rows): asas.trk, asas.tas, asas.vs, asas.asase/asasn (float32). */
int bsa_mvp(bsa_ctx *ctx, const bsa_mvp_params *p,
            const double *gseast, const double *gsnorth, const double *selalt,
            const double *apvs, const uint8_t *noreso, const uint8_t *resooff,
            double *asas_alt, double *trk, double *tas, double *vs,
            float *asase, float *asasn);

/* ---------------------------------------------------------------- kinematics
 * Traffic.UpdateAirSpeed + UpdateGroundSpeed + UpdatePosition
 * (bluesky/traffic/traffic.py:425-483) for n aircraft, one fused kernel.
 * winddim 0 = no wind, 1 = constant wind (windnorth/windeast m/s,
 * windfield.py:150-152), 2 = the context's 2-D wind field (bsa_set_windfield;
 * windnorth/windeast ignored).  Host arrays of length n; state arrays are updated
 * in place; output pointers may be NULL. */
typedef struct bsa_kin_io {
  /* inputs */
  const double *ptas, *phdg, *palt, *pvs; /* pilot.tas/hdg/alt/vs */
  const double *bank, *eps, *accel;       /* traf.bank, traf.eps, perf.acceleration() */
  /* state, in/out */
  double *tas, *hdg, *alt, *vs, *lat, *lon;
  /* outputs */
  double *ax, *delspd, *cas, *mach, *gsnorth, *gseast, *gs, *trk, *coslat, *az;
  uint8_t *swhdgsel, *swaltsel;
} bsa_kin_io;

int bsa_kinematics(bsa_ctx *ctx, int64_t n, double simdt, int winddim,
                   double windnorth, double windeast, bsa_kin_io *io);

/* 2-D wind field for winddim 2 (bsa_kinematics and the resident sim):
 * Windfield.getdata's inverse-distance-squared interpolation
 * (bluesky/traffic/windfield.py:158-179) over nvec definition points at
 * lat/lon [deg] with wind vnorth/veast [m/s] (Windfield.vnorth[0, :] /
 * veast[0, :], as WindSim.addpoint stores them).  Evaluated per aircraft at
 * its pre-step position, for both Pilot.APorASAS (pilot.py:31-35) and
 * UpdateGroundSpeed (traffic.py:463).  Altitude profiles (winddim 3) are not
 * supported: the reference's 3-D branch raises for arrays (windfield.py:177).
 * nvec = 0 clears the field.  Host arrays are copied. */
int bsa_set_windfield(bsa_ctx *ctx, int64_t nvec, const double *lat, const double *lon,
                      const double *vnorth, const double *veast);

/* ---------------------------------------------------------------- geo matrices
 * Standalone materialised producers of
 *   geo.qdrdist_matrix(lat1, lon1, lat2, lon2)      bluesky/tools/geo.py:110-162
 *   geo.kwikqdrdist_matrix(lata, lona, latb, lonb)  bluesky/tools/geo.py:347-363 (BSA_GEO_KWIK)
 * as called outside the CD (traffic/metric.py:596,711,1188 with 1 x m / 1 x n
 * np.matrix operands; traffic/asas/SSD.py:169 with 1-D arrays, i.e.
 * element-wise pairs).  qdr [deg] (KWIK: [0, 360)), dist [nm] (KWIK: metres,
 * as the reference returns them).
 *   outer  (default): out[i*n + j] for i < m, j < n.  qdrdist needs m == n or
 *          m == 1 (its `(lat1 == 0.)*1e-6` term is added to the n-vector
 *          lat2, geo.py:128); KWIK needs m == n (its cavelat is indexed
 *          [j, i], geo.py:355).  Other shapes make the reference broadcast to
 *          a different result shape and are rejected (BSA_EINVAL).
 *   BSA_GEO_PAIRWISE: out[k] for k < m, m == n (1-D operands: every product
 *          of the reference is element-wise).
 * Host arrays are borrowed (float64); qdr / dist are caller-allocated
 * (m*n or m doubles); either may be NULL.  The outputs go through HBM and back
 * over PCIe; bsa_geo_last_ms reports the device time of the producing kernel
 * alone (HIP events on the context stream). */
#define BSA_GEO_KWIK     1
#define BSA_GEO_PAIRWISE 2
int bsa_qdrdist(bsa_ctx *ctx, int64_t m, const double *lat1, const double *lon1,
                int64_t n, const double *lat2, const double *lon2, int flags,
                double *qdr, double *dist);
int bsa_geo_last_ms(bsa_ctx *ctx, double *ms);

/* ---------------------------------------------------------------- multi-GPU
 * One process per GPU, one context per process.  Rank r owns the home rows
 * [r*rpr, min(n, (r+1)*rpr)) of the resident sim, rpr = ceil(n/R) rounded up
 * to a multiple of 512 (a spatially compact chunk of the traffic, SURVEY.md
 * 8e).  Before each CD step every rank receives only the column tiles its rows
 * can reach (a halo exchange: box all-gather, then grouped RCCL send / recv of
 * those tiles' state over xGMI), not the whole state.  No
 * reference equivalent (the reference's only distributed backend,
 * bluesky/network/ ZMQ, is out of scope). */
#define BSA_UNIQUE_ID_BYTES 128
/* Create a communicator id on one rank (ncclGetUniqueId); ship its 128 bytes
 * to the other ranks out of band. */
int bsa_comm_unique_id(char *id128);
int bsa_comm_init(bsa_ctx *ctx, int nranks, int rank, const char *id128);
/* In-process group: several contexts in ONE process form the ranks of a
 * row-sharded sim, each driven by its own host thread, exchanging with
 * device-to-device copies ordered by HIP events (RCCL refuses two ranks on one
 * GPU; this runs the nranks > 1 paths on one GPU and lets one process drive
 * several).  Create the group, then every rank joins it from its thread; the
 * group is freed by bsa_group_destroy once no context is joined any more
 * (destroying it earlier defers the free to its last member's leaving). */
typedef struct bsa_group bsa_group;
bsa_group *bsa_group_create(int nranks);  /* NULL if nranks is not in [1, 16] */
void bsa_group_destroy(bsa_group *g);
int bsa_comm_init_group(bsa_ctx *ctx, bsa_group *g, int rank);
/* Collective: element-wise max of `count` host doubles over all ranks, in
 * place (also a barrier).  Without a communicator it is a no-op. */
int bsa_comm_allreduce_max(bsa_ctx *ctx, double *values, int count);
/* Collective: element-wise sum of `count` host doubles over all ranks. */
int bsa_comm_allreduce_sum(bsa_ctx *ctx, double *values, int count);
/* The communicator as its transport sees it (not collective): info4 =
 * {transport (0 none, 1 RCCL, 2 in-process group), ranks, this rank, device}.
 * With RCCL the ranks / rank / device come from RCCL itself (ncclCommCount,
 * ncclCommUserRank, ncclCommCuDevice), so a report of N ranks is RCCL's. */
int bsa_comm_info(bsa_ctx *ctx, int *info4);

/* C2 pair gather ("pair lists are gathered to the host").
 * Collective over the ranks' last detect (bsa_detect on each rank's row
 * slice, or the resident sim's last CD call): totals3 = {conflict pairs, LoS
 * pairs, rows} summed over all ranks (the root sizes its arrays from them);
 * then bsa_gather_pairs moves every rank's results to `root` and concatenates
 * them in rank order, which is the reference's global row-major order
 * (StateBasedCD.py:93-101) since ranks own contiguous row blocks.  Arrays as
 * in bsa_fetch_pairs (inconf / tcpamax: one entry per row of all ranks); any
 * pointer may be NULL; `out` is read on the root only (dcpa is meaningful
 * only when the detects used BSA_FLAG_WITH_DCPA). */
typedef struct bsa_pairs_out {
  int32_t *ci, *cj;
  double *qdr, *dist, *tcpa, *tinconf, *dcpa;
  int32_t *li, *lj;
  uint8_t *inconf;
  double *tcpamax;
} bsa_pairs_out;
int bsa_gather_counts(bsa_ctx *ctx, int64_t *totals3);
int bsa_gather_pairs(bsa_ctx *ctx, int root, const bsa_pairs_out *out);

/* ---------------------------------------------------------------- GPU-resident sim
 * The synthetic sim step of SURVEY.md 8d with all state resident in HBM:
 *   every cd_every steps: [halo exchange] -> detect (own rows) -> MVP (own rows,
 *                         only if any rank has a conflict, asas.py:486-487)
 *                         -> asas.active = inconf, or (resume_nav = 1) the ASAS
 *                         bookkeeping + ResumeNav (asas.py:409-504) on the device
 *   every step:           Pilot.APorASAS (pilot.py:28-63, winddim 0/1) fused with
 *                         UpdateAirSpeed/GroundSpeed/Position (traffic.py:425-483)
 * AP targets, selalt, bank, eps and perf.acceleration() are frozen inputs.
 * Every array crosses this ABI in aircraft-index order.  On the device the
 * sim keeps them in HOME order (the spatial order of the state at
 * bsa_sim_init): rank r owns the home range [row_begin, row_end) of
 * bsa_sim_stats (512-aligned, spatially compact), whose aircraft indices
 * bsa_sim_row_ids lists; "this rank's rows" below are those aircraft, in
 * ascending index (all of 0..n-1 with one rank). */
typedef struct bsa_sim_params {
  double simdt, rpz, hpz, tla;
  int32_t cd_every; /* >= 1: CD + MVP every k steps (1 = DTNOLOOK=simdt, 20 = asas_dt/simdt) */
  int32_t reso;     /* 1: RESO MVP (MVP.py:14-143); 0: RESO OFF, the reference's default CR
                       (asas.py:41,76-77): DoNothing.resolve (DoNothing.py:11-20) copies the
                       autopilot targets into asas.trk/tas/vs/alt when there are confpairs.
                       Either way asas.active = inconf, or ResumeNav's with resume_nav = 1 */
  bsa_mvp_params mvp;
  int32_t winddim;  /* 0 = no wind, 1 = constant wind (windfield.py:150-152), 2 = 2-D field
                       (bsa_set_windfield): the wind branches of Pilot.APorASAS
                       (pilot.py:31-36,51-61) and UpdateGroundSpeed */
  int32_t resume_nav; /* 1: ASAS.update bookkeeping on the device: resopairs, ResumeNav's
                         asas.active (asas.py:409-471) and the unique / cumulative pair
                         counts (asas.py:490-502); 0: asas.active = inconf */
  double windnorth, windeast; /* [m/s] */
} bsa_sim_params;

typedef struct bsa_sim_state {
  const double *lat, *lon, *alt, *tas, *hdg, *vs, *gs, *trk, *gseast, *gsnorth;
  const double *ap_trk, *ap_tas, *ap_alt, *ap_vs, *selalt, *bank, *eps, *accel;
  const double *asas_alt; /* initial asas.alt (asas.py:405-409 sets it to traf.alt) */
} bsa_sim_state;

typedef struct bsa_sim_out {
  double *lat, *lon, *alt, *tas, *hdg, *vs, *gs, *trk, *gseast, *gsnorth;
  double *asas_trk, *asas_tas, *asas_vs, *asas_alt;
  uint8_t *active;
} bsa_sim_out;

/* Upload the full state (length n, all ranks pass the same) and parameters. */
int bsa_sim_init(bsa_ctx *ctx, int64_t n, const bsa_sim_state *s, const bsa_sim_params *p);
/* Advance nsteps; collective when a communicator is set. */
int bsa_sim_step(bsa_ctx *ctx, int nsteps);
/* Pilot.applylimits with the OpenAP model (pilot.py:65-68 ->
 * performance/openap/perfoap.py:185-209) inside the step, between
 * Pilot.APorASAS and UpdateAirSpeed (traffic.py:397-407): the pilot's tas /
 * vs / alt are clipped to a per-aircraft envelope (full-n host arrays, copied:
 * hmax [m], vmin / vmax [m/s CAS], vsmin / vsmax [m/s], axmax [m/s^2]), the
 * vertical-speed cap scaled by (1 - ax/axmax) with ax = traf.ax of the
 * previous step (0 after bsa_sim_init).  The envelope is a frozen input here;
 * OpenAP's per-phase envelope update (perfoap.py:115-183) is bsa_sim_set_perf,
 * which takes precedence.  hmax == NULL switches the limits off (the default
 * after bsa_sim_init). */
int bsa_sim_set_limits(bsa_ctx *ctx, const double *hmax, const double *vmin, const double *vmax,
                       const double *vsmin, const double *vsmax, const double *axmax);
/* OpenAP.update (performance/openap/perfoap.py:115-131) inside the step:
 * each aircraft's flight phase is inferred from its pre-step vs / alt
 * (phase.py:14-62), its envelope looked up in its type's row at that phase
 * (__construct_limit_matrix, perfoap.py:211-262) and applied as
 * bsa_sim_set_limits does, and UpdateAirSpeed's acceleration is
 * OpenAP.acceleration() (2 m/s^2 in phase GD, else 0.5; perfoap.py:271-280)
 * instead of the frozen accel.  table: ntypes rows of 24 doubles -- vmin by
 * phase NA..GD (9), vmax by phase (9), vsmin, vsmax, hmax, axmax, lifttype
 * (1 fixed wing, 2 rotor, 0 other), 0 (bluesky_amd/perf.py builds it from the
 * reference's Coefficient tables); type_idx: full-n row per aircraft
 * (validated).  Takes precedence over bsa_sim_set_limits; table == NULL
 * switches it off (the default after bsa_sim_init). */
int bsa_sim_set_perf(bsa_ctx *ctx, int64_t ntypes, const double *table, const int32_t *type_idx);
/* This rank's rows of the flight phase of the last step
 * (0..8, phase.py:4-12; needs bsa_sim_set_perf) and of traf.ax, written into
 * full-n host arrays; either pointer may be NULL. */
int bsa_sim_read_perf(bsa_ctx *ctx, uint8_t *phase, double *ax);
/* Traffic.update's atmosphere, traf.p / rho / Temp = vatmos(traf.alt) on the
 * pre-step altitude (traffic.py:389, aero.py:62-74), computed inside the step
 * when on (off after bsa_sim_init: nothing in the step reads them; a host
 * performance model in hybrid mode does).  _read: this rank's rows of the last
 * step into full-n host arrays [Pa, kg/m3, K]; any pointer may be NULL. */
int bsa_sim_set_atmos(bsa_ctx *ctx, int on);
int bsa_sim_read_atmos(bsa_ctx *ctx, double *p, double *rho, double *temp);
/* Overwrite per-aircraft arrays of the resident sim (full-n host arrays, all
 * ranks pass the same) while keeping the ASAS bookkeeping (resopairs, the
 * previous call's pair sets, asas.active / trk / tas / vs) and traf.ax: the
 * hybrid mode where the host simulator (autopilot, performance model, stack
 * commands) changes traffic between steps (traffic.py:383-404 runs them
 * before Traffic.update's kinematics).  NULL pointers leave that array as it
 * is; asas_alt overwrites the persistent asas.alt. */
int bsa_sim_update(bsa_ctx *ctx, const bsa_sim_state *s);
/* Traffic.create for the resident sim (traffic.py:192-312 + ASAS.create,
 * asas.py:402-407): append m aircraft whose state is s (m-long host arrays,
 * every field required); asas.trk / tas start at trk / tas, asas.alt at
 * s->asas_alt, asas.vs / active / traf.ax at 0.  They take indices n..n+m-1.
 * Fails while OpenAP limits are on (set them again after).  Collective with
 * several ranks (all pass the same arrays): every rank's replicas are completed
 * first, the rows re-partitioned over the new n afterwards (each rank keeps
 * the bookkeeping of its new range). */
int bsa_sim_create(bsa_ctx *ctx, int64_t m, const bsa_sim_state *s);
/* Traffic.delete for the resident sim (traffic.py:364-378 ->
 * trafficarrays.py:99-117): remove the k aircraft idx[0..k) (any order,
 * duplicates ignored); the rest keep their order and shift down, as np.delete
 * does.  The ASAS bookkeeping follows the reference's callsign-keyed sets:
 * resopairs of a deleted ownship go; a resopair whose intruder was deleted
 * stays (bsa_sim_resopairs reports idx2 = -1) until the next CD call's
 * ResumeNav switches the ownship's ASAS off and drops it (asas.py:419-468).
 * Removing every aircraft is an error (re-init instead).  Collective with
 * several ranks (all pass the same list), re-partitioned as bsa_sim_create. */
int bsa_sim_delete(bsa_ctx *ctx, int64_t k, const int64_t *idx);
/* Full-n host copies of the state (collective: gathers all ranks' rows).
 * Any pointer may be NULL. */
int bsa_sim_read(bsa_ctx *ctx, bsa_sim_out *o);
/* [0] steps done, [1] CD calls, [2] conflicts and [3] LoS pairs of the last
 * CD call (this rank's rows), [4] this rank's row_begin, [5] row_end (its home
 * range: row_end - row_begin rows; (0, n) with one rank). */
int bsa_sim_stats(bsa_ctx *ctx, int64_t *out6);
/* The aircraft indices of this rank's rows, ascending (row_end - row_begin
 * entries): the rows of bsa_sim_acdata_poll's arrays, of bsa_fetch_pairs'
 * inconf / tcpamax after resident steps, and of bsa_sim_read_perf. */
int bsa_sim_row_ids(bsa_ctx *ctx, int32_t *ids);
/* Measurement aid: the sim's detect (home order, its rpz / hpz / tla) of the
 * home rows [row_begin, row_end) (row_begin a multiple of 512) against all
 * columns -- one rank's share of a CD step, on one GPU, as that rank computes
 * it: its own column tiles, the halo plan, the halo tiles (bsa_sim_halo_stats
 * [2] counts them; the boxes of all tiles, which the other ranks would send,
 * are prepared before the timed stages).  Its pairs REPLACE the
 * last CD call's as the fetchable / gatherable pairs (bsa_fetch_pairs); the
 * sim's state and ASAS bookkeeping are not changed, and the next CD step
 * detects the sim's own rows again. */
int bsa_sim_detect_rows(bsa_ctx *ctx, int64_t row_begin, int64_t row_end, int64_t *n_conf, int64_t *n_los);
/* Halo exchange of the sharded step (several ranks): [0] bytes
 * this rank receives and [1] sends per CD call (the agreed capacities' regions),
 * [2] column tiles (512 aircraft) it received at the last CD call -- or, after
 * bsa_sim_detect_rows, the tiles that rank share needs from other ranks --
 * and [3] capacity regrowths (aborted and re-run steps) since bsa_sim_init. */
int bsa_sim_halo_stats(bsa_ctx *ctx, int64_t *out4);
/* Stream-ordered collectives (RCCL or the in-process group) this rank issued
 * since the last bsa_timing_reset: [0] calls, [1] payload bytes it sent,
 * [2] payload bytes it received (as RCCL moves them).  Per CD step of the
 * sharded sim: the box all-gather, the halo send / recv, the 16-B gate
 * all-reduce (+ the pair-key all-gather with resume_nav). */
int bsa_sim_comm_stats(bsa_ctx *ctx, int64_t *out3);
/* Testing aid: override this rank's copy of the tile capacity sender ->
 * receiver (the capacities must agree on all ranks, and RCCL's grouped send /
 * recv needs every send length to match its receive; the in-process group
 * checks that agreement at every exchange and fails loudly, so a disagreement
 * is caught on one GPU).  tiles >= 0; the next bsa_sim_init or regrowth
 * recomputes the capacities. */
int bsa_sim_set_halo_cap(bsa_ctx *ctx, int sender, int receiver, int64_t tiles);
/* Measurement aid (tools/probe_step.py): a ONE-rank sim plays rank `rank` of
 * `nranks` on this GPU -- bsa_sim_step then runs that rank's share of the
 * sharded step (its home rows: own tiles, halo plan and halo tiles as
 * bsa_sim_detect_rows does, K3 / K4' on its rows) with no collective; the
 * other rows do not move.  The results are not the sim's (timing only);
 * nranks = 1 returns to the whole sim (re-init it for results). */
int bsa_sim_probe_rank(bsa_ctx *ctx, int rank, int nranks);
/* Collective (every rank, before the same step): the next halo exchange
 * re-checks the region layout on all ranks -- every send length / offset
 * against its receiver's expectation, one host all-reduce -- as it does after
 * bsa_sim_init and every capacity regrowth, before any RCCL send / recv is
 * enqueued; a disagreement fails the step on every rank ("halo lengths
 * disagree").  Testing aid with bsa_sim_set_halo_cap. */
int bsa_sim_halo_recheck(bsa_ctx *ctx);
/* ASAS bookkeeping after the last CD call (resume_nav = 1; replaces
 * ASAS.update's Python sets, asas.py:490-502):
 * [0] |resopairs| of this rank's rows, [1] |confpairs_unique|,
 * [2] |lospairs_unique|, [3] len(confpairs_all), [4] len(lospairs_all),
 * [5] number of active aircraft of this rank's rows.  [1]-[4] are counts of
 * the global pair sets (every rank gathers all ranks' pair keys; the same
 * values on every rank). */
int bsa_sim_asas_stats(bsa_ctx *ctx, int64_t *out6);
/* This rank's resopairs (aircraft indices; idx1 ascending, then idx2; idx2 = -1, last in its
 * row, for an intruder deleted since the last CD call), at most cap pairs;
 * *count = total (call again with a larger buffer when *count > cap). */
int bsa_sim_resopairs(bsa_ctx *ctx, int32_t *idx1, int32_t *idx2, int64_t cap, int64_t *count);

/* One CD call of the resident sim WITHOUT the kinematics: [halo exchange] ->
 * detect -> resolver -> asas.active or the bookkeeping + ResumeNav, i.e. the
 * body of ASAS.update (asas.py:478-504), exactly the CD part of a
 * bsa_sim_step; the state does not move and the step count does not advance.
 * The ASAS.update drop-in (bluesky_amd/asas.py) runs it after writing the host
 * simulator's traffic with bsa_sim_update.  Overflows are grown and re-run
 * inside the call.  Collective with several ranks. */
int bsa_sim_cd(bsa_ctx *ctx);
/* Replace the parameters of a running sim (stack commands such as ZONER,
 * ZONEDH, DTLOOK, RMETHH change asas.R / dh / dtlookahead / the MVP switches
 * between calls, asas.py:190-395).  Turning resume_nav on starts with empty
 * bookkeeping. */
int bsa_sim_set_params(bsa_ctx *ctx, const bsa_sim_params *p);
/* NORESO / RESOOFF lists (asas.noresolst / asas.resoofflst, MVP.py:44-61) as
 * full-n uint8 host arrays of membership in aircraft-index order (NULL = empty
 * list); the step's MVP applies them when mvp.swnoreso / swresooff are set.
 * They follow bsa_sim_delete / bsa_sim_create (new aircraft are in neither). */
int bsa_sim_set_reso_lists(bsa_ctx *ctx, const uint8_t *noreso, const uint8_t *resooff);
/* ASAS outputs of this rank's rows after the last CD call, written into
 * full-n host arrays (other rows untouched; any pointer may be NULL):
 * asas.trk / tas / vs / alt, asase / asasn (float32), asas.active, and
 * dropped = 1 for an ownship of which ResumeNav dropped a resopair in that call
 * (asas.py:454-468: the reference then starts waypoint recovery with
 * route.direct, which is autopilot state the host applies; resume_nav = 1). */
typedef struct bsa_asas_out {
  double *trk, *tas, *vs, *alt;
  float *asase, *asasn;
  uint8_t *active, *dropped;
} bsa_asas_out;
int bsa_sim_read_asas(bsa_ctx *ctx, bsa_asas_out *o);

/* ACDATA feed: the per-aircraft fields
 * ScreenIO.send_aircraft_data streams at 5 Hz
 * (bluesky/simulation/qtgl/screenio.py:194-239) for this rank's rows, served
 * from HBM without stalling the sim.  _request enqueues a snapshot behind the
 * steps already queued (one pack kernel + one copy into a pinned host mirror;
 * no host synchronisation); _poll returns 1 while it is still in flight (wait
 * = 0) or waits for it (wait = 1), then copies it into the caller's arrays
 * (row_end - row_begin entries each; any pointer may be NULL) and returns 0.
 * inconf / tcpamax are asas.inconf / asas.tcpamax of the last CD call (0
 * before the first), cas is traf.cas after the last step (0 before the first),
 * asasn / asase as asas holds them.  nconf_cur / nlos_cur = len(confpairs_unique) /
 * len(lospairs_unique), nconf_tot / nlos_tot = len(confpairs_all) /
 * len(lospairs_all) (screenio.py:207-210), global over all ranks; -1 unless
 * resume_nav = 1.  A new request first waits for the previous snapshot. */
typedef struct bsa_acdata {
  int64_t steps, row_begin, row_end;  /* set by _poll */
  int64_t nconf_cur, nconf_tot, nlos_cur, nlos_tot;
  double *lat, *lon, *alt, *tas, *cas, *gs, *trk, *vs, *tcpamax;
  uint8_t *inconf;
  float *asasn, *asase;
} bsa_acdata;
int bsa_sim_acdata_request(bsa_ctx *ctx);
int bsa_sim_acdata_poll(bsa_ctx *ctx, int wait, bsa_acdata *out);

#ifdef __cplusplus
}
#endif
#endif /* BSACCEL_H */
