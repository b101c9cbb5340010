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
 * Any pointer may be NULL to skip that output. */
int bsa_fetch_pairs(bsa_ctx *ctx,
                    int32_t *ci, int32_t *cj, double *qdr, double *dist,
                    double *tcpa, double *tinconf, double *dcpa,
                    int32_t *li, int32_t *lj,
                    uint8_t *inconf, double *tcpamax);

/* Candidate-pair count of the last detect (pairs that passed the
 * conservative prefilter and were evaluated exactly in fp64). */
int bsa_last_candidates(bsa_ctx *ctx, int64_t *n_candidates);

/* Tile pairs (512 rows x 512 columns) of the last detect that survived the
 * bounding-box cull, and the total number of tile pairs. */
int bsa_last_tiles(bsa_ctx *ctx, int64_t *kept, int64_t *total);

/* Device time of the last detect's stages in milliseconds, measured with
 * HIP events on the context stream: [0] spatial order + records + tile cull,
 * [1] prefilter, [2] exact, [3] sort+gather, [4] whole detect. */
int bsa_last_timings(bsa_ctx *ctx, double *ms5);

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
 * windfield.py:150-152).  Host arrays of length n; state arrays are updated
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

#ifdef __cplusplus
}
#endif
#endif /* BSACCEL_H */
