// Internal runtime of libbsaccel: context, device buffers, error plumbing.
// gfx950 (MI355X) only; compiled with -ffp-contract=off so every fp64
// expression rounds exactly like numpy's (one rounding per operation).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/bsaccel.h"

namespace bsa {

// ---------------------------------------------------------------- constants
// bluesky/tools/aero.py:11-28, bluesky/tools/geo.py:7,38-39
constexpr double kNM = 1852.0;
constexpr double kFT = 0.3048;
constexpr double kKTS = 0.514444;
constexpr double kWGS84_A = 6378137.0;
constexpr double kWGS84_B = 6356752.314245;
constexpr double kPI = 3.14159265358979323846;  // NPY_PI
constexpr double kD2R = kPI / 180.0;            // numpy deg2rad / radians factor
constexpr double kR2D = 180.0 / kPI;            // numpy rad2deg / degrees factor

// ---------------------------------------------------------------- records
// Per-index fp64 records gathered by the exact pair kernel (128 B = one
// cache line each).  Orientation follows StateBasedCD.py: for pair (i, j)
// the geometry row is ownship i and the column is intruder j, while the
// velocity / altitude differences are own[j] - intruder[i]
// (StateBasedCD.py:39-40,65-69).  So the ROW record i carries own[i]'s
// position and intruder[i]'s velocity; the COLUMN record j carries
// intruder[j]'s position and own[j]'s velocity.
struct alignas(16) RowRec {
  double lat, lon;        // own[i] [deg]
  double sinlat, coslat;  // sin/cos(radians(own.lat[i]))          geo.py:137-140
  double hemA;            // |lat| * (rwgs84(lat) + a)              geo.py:127
  double u, v;            // int.gs[i] * sin/cos(radians(int.trk[i]))  StateBasedCD.py:35-37
  double alt, vs;         // int.alt[i], int.vs[i]
  double pad0;
  double ilat;            // int.lat[i]  (KWIK cavelat, geo.py:355; same offset as ColRec::olat)
  double pad[5];
};
struct alignas(16) ColRec {
  double lat, lon;        // int[j]
  double sinlat, coslat;
  double hemA;
  double u, v;            // own.gs[j] * sin/cos(radians(own.trk[j]))  StateBasedCD.py:30-32
  double alt, vs;         // own.alt[j], own.vs[j]
  double eps;             // (own.lat[j] == 0.) * 1e-6                geo.py:128
  double olat;            // own.lat[j]  (KWIK cavelat, geo.py:355)
  double pad[5];
};
static_assert(sizeof(RowRec) == 128, "RowRec must be one cache line");
static_assert(sizeof(ColRec) == 128, "ColRec must be one cache line");

// fp32 prefilter record (32 B), one per sorted row / column.
// Stage 1 keeps a pair iff |x_i - x_j| < s_i + s_j (tested in a plane, see
// k_prefilter) and lo_j < hi_i and hi_j > lo_i (<=> |a_j - a_i| < h_i + h_j).
// x / a are the position / altitude at t = 0, or (midpoint mode, DESIGN.md
// 3.2b) at t = tla/2 along the velocity, with the reaches to match.
struct alignas(16) PFRec {
  float x, y, z;   // stage-1 point (unit-sphere units)
  float s;         // horizontal reach, chord units (half of the pair bound); INF = always
  float lo, hi;    // a -/+ h, h = vertical reach [m] (half of the pair bound)
  float alt;       // altitude [m] at t = 0 (refine)
  float pad;
};
// The refine's position (PFPos, float4 x y z 0): the unit vector at t = 0.
static_assert(sizeof(PFRec) == 32, "PFRec must be 32 B");

// velocity part, read only by the CPA refine (rows and columns)
struct alignas(16) PFVel {
  float u, v;      // east / north velocity [m/s] (orientation as RowRec / ColRec)
  float vs;        // vertical speed [m/s]
  unsigned flags;  // bit 0: never refine this index (unbounded radius quirk / non-finite
                   //        / tangent basis ill-conditioned near a pole)
};
static_assert(sizeof(PFVel) == 16, "PFVel must be 16 B");

// Candidate-list reuse (BSA reuse mode): state of one
// aircraft (sorted position) when the candidate list was last built, and its
// vertical budget [m].  The unit vector and velocity are fp64.
struct alignas(16) Snap {
  double x, y, z;   // unit position vector
  double u, v;      // gs * sin / cos(trk)
  double alt, vs;
  float sv;         // vertical budget of this build [m]
  float pad;
};
static_assert(sizeof(Snap) == 64, "Snap must be 64 B");

// axis-aligned bounds of a group / tile of sorted PFRecs (culling)
struct alignas(16) TileBox {
  float lo[3], hi[3];   // unit-vector bounds
  float vlo, vhi;       // min lo, max hi (vertical reach intervals)
  float smax, pad0;
  int count, pad1;
};
static_assert(sizeof(TileBox) == 48, "TileBox must be 48 B");

constexpr int kTile = 512;  // rows per row block == columns per column tile
constexpr int kResortEvery = 8;  // detect calls between spatial re-sorts
constexpr int kResortEveryReuse = 64;  // ... with a reusable candidate list (a re-sort rebuilds it)
constexpr int kEvSets = 4096;    // detect timing event sets kept between resets

#ifndef BSA_CAND_SHARDS
#define BSA_CAND_SHARDS 8
#endif
constexpr int kCandShards = BSA_CAND_SHARDS;  // candidate list shards (one counter each, 128 B apart)
constexpr unsigned kDangling = 0xffffffffu;  // resopairs column of a deleted intruder (sorts last in a row)
// gate[0] of the resident step (all-reduced max over ranks): 0 nothing, 1 a
// non-finite tcpa input in some rank's columns (every row's tcpamax is NaN),
// >= 2 abort the step (2 candidate / row-bucket overflow, 3 resopairs overflow)
constexpr unsigned long long kGateNonfinite = 1, kGateOverflow = 2, kGateBkOverflow = 3;
// gate[2]: the HK prediction of this CD call (some rank's records left kHkPredict of their budgets)
constexpr int kGateWords = 3;
constexpr int kSimCtlSticky = 24, kSimCtlSteps = 32, kSimCtlDemand = 40, kSimCtlKdemand = 48, kSimCtlStale = 56;
// (sim_ctl bytes; [24, 64) are zeroed per batch and read back after it)
constexpr int kHkRing = 16;  // HK: published predictions (pinned host words), slot m % kHkRing
constexpr unsigned long long kNanBits = 0x7ff8000000000000ull;  // (a quiet NaN)

// HK publication (Ctx::hk_*): lane 0 of block 0 of a CD step's K4' (or of the
// fused K2 + K4') stores base | prediction (bit 0) | aborted (bit 1) into the
// ring slot of the detect, in pinned host memory the host polls (a vector
// store, system scope; written before any early return of the kernel)
struct HkPub {
  unsigned long long *slot;  // device view of hk_host[m % kHkRing], or NULL (no publication)
  unsigned long long base;   // (m + 1) << 2
  unsigned long long *src;   // the prediction word (gate[2] after the all-reduce, or the rank's own word)
  int zero;                  // zero *src once read (the rank's own word: its next user is two detects on)
};
// (relaxed: the host reads this one word; a release at system scope would
// write back the whole L2 first -- buffer_wbl2 -- under the other waves' feet)
template <typename Aborted>
__device__ __forceinline__ void hk_publish(const HkPub &p, Aborted aborted) {
  if (!p.slot) return;
  const unsigned long long v = p.base | (p.src && *p.src ? 1ull : 0ull) | (aborted() ? 2ull : 0ull);
  if (p.zero && p.src) *p.src = 0ull;
  __hip_atomic_store(p.slot, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// counters block on the device
constexpr int kFuseRecsMax = 64;  // fused K1b: mid-sweep flush records per prefilter wave (LDS)

struct Counters {
  unsigned long long cand;    // host-side total (sum of the shard counts)
  unsigned long long conf;
  unsigned long long los;
  unsigned long long tiles;
  unsigned long long groups;  // (64-row x 8-column) blocks swept by the prefilter
  unsigned long long tiles_near;  // of `tiles`: pairs whose boxes overlap (listed first, swept first)
  unsigned long long tpr_stale;   // a host-kept tile-pair list (HK) whose records left their budgets: re-run
  unsigned long long k2_demand;   // K2 row buckets: the largest row count beyond Ctx::k2_bucket (0: fit)
  unsigned long long halo_ovf;    // halo exchange: more tiles to send / receive than the capacities
  unsigned long long halo_miss;   // halo exchange inconsistent (a kept tile pair without its data): bug
  unsigned long long fuse_ovf;    // fused K1b: a wave flushed more blocks than it can record (retry unfused)
  // diagnostic builds only (-DBSA_PF_STAMPS): prefilter s_memtime cycles per phase
  unsigned long long stamp[8];
  unsigned long long cshard[kCandShards][16];  // candidates per shard (word 0 of each line)
  unsigned long long gpart[32][16];  // sub-groups swept, per prefilter workgroup shard (summed into groups by K2)
};

// ---------------------------------------------------------------- buffers
struct DevBuf {
  void *p = nullptr;
  size_t bytes = 0;
};

struct Ctx;
bool ensure(Ctx *c, DevBuf &b, size_t bytes, const char *what);
// Pinned host staging (bsa_ctx.hip): host_copy copies its jobs with a small
// thread pool (chunks of 256 KiB; small totals on the calling thread);
// pin_stage returns the context's pinned buffer of >= bytes once no DMA from
// it is pending; pin_issued marks a DMA from it just enqueued on c->stream.
struct HostCopy {
  void *dst;
  const void *src;
  size_t bytes;
};
void host_copy(const HostCopy *jobs, int n);
constexpr int kGatherMax = 12;
struct GatherParts {
  const unsigned *src[kGatherMax];
  unsigned long long woff[kGatherMax + 1];
  unsigned long long wlen[kGatherMax];
  int n;
};
__global__ void k_gather_words(GatherParts g, unsigned *__restrict__ dst);
unsigned char *pin_stage(Ctx *c, size_t bytes);
int pin_issued(Ctx *c);
bool ensure_keep(Ctx *c, DevBuf &b, size_t bytes, const char *what);  // grows, keeps contents
void release(DevBuf &b);

struct Ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;

  // state
  int64_t n = 0;
  bool has_intruder = false;
  DevBuf own[6];   // lat lon trk gs alt vs
  DevBuf intr[6];
  DevBuf rowrec, colrec, pfrow, pfcol, pfvrow, pfvcol, pfprow, pfpcol;
  // spatial order: Morton keys and the sorted-position -> original-index maps
  DevBuf key_r, idx_r, key_r2, perm_r, key_c, idx_c, key_c2, perm_c;
  DevBuf tbox_r, tbox_c, gbox_r, gbox_c, sbox_c, tilepairs, workq;
  DevBuf rowcnt, rowoff;         // K2 counting sort
  DevBuf kbuck;                  // K2 row buckets (column indices)
  int k2_bucket = 8;             // bucket width (pairs per row); 0 = scatter into row segments
  DevBuf scan_ws;                // single-pass scan: [0] ticket counter, then tile status words
  bool scan_ready = false;
  unsigned long long scan_tickets = 0;
  unsigned scan_epoch = 0;
  // reusable spatial order (any permutation gives identical results)
  bool perm_valid = false, perm_shared = false, perm_distinct = false;
  double perm_f = 0.0;  // midpoint factor the spatial order was computed with (k_keys)
  int64_t perm_n = 0, perm_rb = 0, perm_re = 0, perm_age = 0;

  // detect buffers
  DevBuf counters;           // Counters
  DevBuf counters2, workq2;  // the next detect's counters / dequeue words (double-buffered, zeroed by K2)
  int64_t zeroed_rows = -1;  // rows of the last detect whose K2 zeroed counters2 / workq2 / rowcnt, or -1
  DevBuf cand;               // uint2 (i, j)
  DevBuf cflag;              // per candidate: bit0 conflict, bit1 LoS
  unsigned long long cand_cap = 0;
  DevBuf ckey, cval, ckey2, cval2;  // conflict keys / slot ids (+ sorted)
  DevBuf cpay;               // 5 x cap doubles: qdr dist tcpa tin dcpa (slot order)
  unsigned long long conf_cap = 0;
  DevBuf lkey, lkey2;        // LoS keys (+ sorted)
  unsigned long long los_cap = 0;
  DevBuf out_ci, out_cj, out_li, out_lj;  // int32 sorted
  DevBuf out_pay;            // 5 x n_conf doubles, sorted
  DevBuf inconf, tcpamax;    // per row of the last detect
  DevBuf sort_tmp;

  // last detect
  int64_t last_rb = 0, last_re = 0;
  int64_t last_conf = 0, last_los = 0, last_cand = 0, last_tiles = 0, last_tiles_total = 0,
          last_groups = 0;
  int last_flags = 0;
  bool have_pairs = false;

  // candidate-list reuse across detects (shared own == intruder only)
  bool reuse_on = false;
  double reuse_sh = 800.0, reuse_sv = 60.0;   // horizontal budget, default / max vertical budget [m]
  bool reuse_valid = false;                   // a list + snapshot exist for the current perm / params
  double reuse_key[4] = {0, 0, 0, 0};         // rpz hpz tla flags of the list
  int64_t reuse_n = -1;
  unsigned long long reuse_cap = 0;
  void *reuse_candp = nullptr;
  DevBuf snap_build, snap_cur, reuse_ctl, reuse_use;  // ctl: [0] build flag, [1] detects since build

  // tile-pair list reuse: K0d's item list, built on boxes
  // inflated by (tpr_dx chord, tpr_ds reach, tpr_dv m), is kept while every
  // aircraft's prefilter record stays within those distances of its record at
  // the build (checked by whoever prepares the records: K4' / K0b); a record
  // outside raises tpr_ctl[0] and the next detect rebuilds on the device
  bool tpr_on = true;                  // resident home-order detects of all rows (BSA_TPR=0: off)
  bool tpr_valid = false;              // a list + snapshot exist for tpr_key / tpr_n
  double tpr_key[6] = {0, 0, 0, 0, 0, 0};  // rpz hpz tla mid row_begin row_end of the list
  int64_t tpr_n = -1;
  float tpr_dx = 3.2e-4f, tpr_ds = 1.6e-5f, tpr_dv = 300.f;  // ~2 km, ~100 m of reach, 300 m
  DevBuf tpr_snap;                     // PFRec per aircraft at the last build
  DevBuf tpr_ctl;                      // u64: [0] build flag, [1] near items, [2] far items, [3] builds, [4] detects,
                                       // [5] the probe's rebuild flag, [6 + (m & 1)] HK prediction of detect m
  // Host-known list decisions (HK, round 6): in the resident
  // step the host decides build / keep BEFORE it enqueues a detect, so a kept
  // list launches no K0d (and, several ranks, no box all-gather, no halo plan
  // and one K0b for own + halo tiles).  Detect m keeps when neither m-1 nor
  // m-2 built and the device's prediction for m -- the records of detect m-2
  // within kHkPredict of every budget, over all ranks -- says so; the step's
  // K4' publishes that prediction into a pinned host ring (hk_host), so the
  // host waits at most for the work of the step before.  The kept detect still
  // checks every record against the full budgets: one outside aborts the step
  // (Counters::tpr_stale) and it re-runs with a build.
  bool hk_on = true;                   // BSA_HK=0: the device decides (round-5 behaviour)
  bool hk_req = false;                 // bsa_sim_step: the detect being enqueued may be host-decided
  bool hk_ok = false;                  // the build history below is this sim's
  bool hk_built[4] = {false, false, false, false};  // build decisions of detects m & 3
  bool hk_cur = false, hk_keep = false;  // the last detect_enqueue was host-decided / kept its list
  int64_t hk_m = 0;                    // index of the next host-decided detect
  int64_t hk_last = 0;                 // ... of the last one (its K4' publishes slot hk_last % kHkRing)
  int64_t hk_cool = 0;                 // after a stale abort: device-decided detects left
  int64_t hk_cool_len = 32;            // ... the next such stretch (doubles per stale abort, <= 4096):
                                       // a workload whose lists go stale often ends up device-decided
  int64_t hk_keeps = 0, hk_builds = 0, hk_stale = 0, hk_waits = 0;  // statistics
  float hk_f = 0.75f;                  // prediction fraction of the budgets (BSA_HK_F)
  unsigned long long *hk_host = nullptr, *hk_hdev = nullptr;  // pinned ring (host / device view)
  // longest items first (bsa_cd.hip HeavyArgs): per list slot cost / flag, two item lists and counts
  DevBuf hv_cost, hv_flag, hv_list[4], hv_cnt;  // lists: [parity][tier]
  unsigned long long hv_icap = 0;
  unsigned hv_epoch = 0;
  double hv_us = 16.0;                 // listing threshold [us] per item (BSA_PF_HEAVY_US at bsa_create; < 0: off)
  bool hv_us_env = false;              // ... set by BSA_PF_HEAVY_US (else halved for a rank's share, bsa_cd.hip)
  double hv_x = 3.0;                   // ... x this: the top tier, twice the pieces (BSA_PF_HEAVY_X; <= 0: one tier)
  // halo overlap (round 6): on a kept-plan detect of several
  // ranks the halo send / recv, the halo K0b and the sweep of the halo column
  // tiles run on xstream while the own tiles' K0b and sweep run on `stream`;
  // joined by ov_ev[2] before K1b.  ov_mode: 1 exchange mode only (default),
  // 2 also the one-GPU probe (its cost without an exchange to hide), 0 off
  // (BSA_HALO_OVERLAP at bsa_create).  Off by default: on one GPU the split
  // costs ~17 us per step (probe, no exchange to hide: two sweeps' ramps and
  // tails + cross-stream event waits of ~5-10 us each), more than the ~30 us
  // exchange it could hide would repay only on the 8-GPU node
  int ov_mode = 0;
  hipStream_t xstream = nullptr;
  hipEvent_t ov_ev[3] = {nullptr, nullptr, nullptr};  // packed / own tiles prepared / halo sweep done
  int64_t ov_count = 0;                // overlapped detects (statistics)
  // (device-scope events: the join's wait 13 -> 10 us, the step 0.136 -> 0.134 ms; BSA_OV_EVFLAGS, A/B)
  unsigned ov_evflags = hipEventDisableTiming | hipEventDisableSystemFence;

  // detect timing: one set of 5 events per detect since the last reset
  std::vector<hipEvent_t> evpool;
  int ev_sets = 0, ev_last = 0;
  int ev_every = 1;       // time one detect in ev_every (0 = none), bsa_set_timing_sample
  int64_t ev_count = 0;   // detects since the last bsa_timing_reset
  bool ev_valid = false;
  bool empty_detect = false;
  DevBuf stats;  // accumulated per-detect statistics {groups, candidates, tiles, detects, list builds}
  void *trace_buf = nullptr;  // diagnostic builds (-DBSA_PF_TRACE): prefilter item timeline
  size_t trace_bytes = 0;

  // MVP / kinematics staging (host-buffer entry points)
  DevBuf seg, mvp_stage, kin_stage, mvp_pdv, mvp_pfl, mvp_rowdv;
  DevBuf xfer_stage;  // batched home-order transfers (bsa_sim.hip: HomeBatch), index-order staging
  // pinned host staging of the drop-ins' transfers (pin_stage, bsa_ctx.hip):
  // one DMA per batch; pin_ev guards the buffer while a DMA from it may run
  void *pin = nullptr;
  size_t pin_bytes = 0;
  hipEvent_t pin_ev = nullptr;
  bool pin_busy = false;

  // multi-GPU: comm is an ncclComm_t (one process per GPU) or group an
  // in-process group of contexts (bsa_comm.hip); at most one is set
  void *comm = nullptr;
  struct Group *group = nullptr;
  int nranks = 1, rank = 0;
  DevBuf red;  // small reduction scratch
  // stream-ordered collectives this rank issued since the last bsa_timing_reset
  // (bsa_sim_comm_stats): calls and the bytes it sends / receives (payload,
  // as RCCL would move them; the in-process group's staging copies aside)
  int64_t comm_calls = 0, comm_tx = 0, comm_rx = 0;
  DevBuf pg_send, pg_recv;  // C2 pair gather staging (bsa_gather_pairs)

  // GPU-resident sim (bsa_sim.hip).  Its state lives in HOME order: home
  // position h holds aircraft h2id[h] (id2h is the inverse), fixed at init as
  // the spatial order of the initial traffic, so a rank's rows are a
  // contiguous, spatially compact home range [sim_rb, sim_re) (512-aligned)
  // and the detect reads its columns without a gather or a re-sort.  lpos[r]:
  // position of home sim_rb + r among the rank's rows sorted by aircraft index.
  bool home = false;                  // own[] and the sim arrays are in home order
  bool det_home = false;              // detect_enqueue: home-ordered state (set by sim_cd)
  bool last_home = false;             // the last detect's ci / li are home rows (fetch translates)
  DevBuf h2id, id2h;                  // u32, device
  DevBuf lbyidx;                      // u32, device: this rank's home rows (relative) in ascending index order
  DevBuf fetch_stage;                 // fetch_pairs of a home-order detect: the lists re-ordered on the device
  std::vector<unsigned> h2id_h, id2h_h, lpos_h;  // host copies
  bool sim_ready = false;
  bool mvp_deferred = false;            // this step's K3 rows run inside K4' (sim_cd -> bsa_sim_step)
  std::vector<unsigned char> mvp_defer;  // the deferred K3 arguments (MvpIn, bsa_mvp_row.h)
  // K2 fused with K4' (one rank): sim_cd asks (k24_want), detect_enqueue then
  // keeps its K2 launch (k24_blob) for k24_launch, with the timed detect's
  // last stage event; alt / vs / gseast / gsnorth double buffers
  bool k24_want = false, k24_pending = false;
  std::vector<unsigned char> k24_blob;
  hipEvent_t k24_ev = nullptr;
  DevBuf nx_alt, nx_vs, nx_gse, nx_gsn;
  bsa_sim_params simp{};
  int64_t sim_steps = 0, sim_cd_calls = 0, sim_rb = 0, sim_re = 0, sim_rpr = 0;
  int64_t sim_last_conf = 0, sim_last_los = 0;
  bool sim_gathered = true;  // replicas consistent with every rank's rows
  bool sim_gs_derivable = false;  // gseast / gsnorth of every row follow from gs / trk (K4' without wind ran)
  bool sim_prepped = false;       // the last K4' wrote the next detect's column records / boxes (one rank)
  double sim_prep_key[4] = {0, 0, 0, 0};  // ... for rpz, hpz, tla, stage-1 mode
  int64_t sim_prep_n = 0;
  DevBuf s_tas, s_hdg, s_gse, s_gsn;                        // traffic state besides own[]
  DevBuf s_aptrk, s_aptas, s_apalt, s_apvs, s_selalt, s_bank, s_eps, s_accel;  // frozen
  DevBuf s_atrk, s_atas, s_avs, s_aalt, s_ase, s_asn, s_active;  // ASAS (full n)
  DevBuf g_send, g_recv;                                    // all-gather staging
  // Non-finite tcpa inputs (StateBasedCD.py:90: tcpamax = np.max(tcpa *
  // swconfl) is NaN on every row once one tcpa is NaN): nonfin[0] = the epoch
  // of the last column records holding a non-finite lat / lon / u / v (its
  // producers store the epoch, K2 compares; no zeroing, no atomics)
  DevBuf nonfin;
  DevBuf rownf;  // rows of their own (not columns): per row (index order), its position / velocity is not finite
  unsigned long long nf_counter = 0, nf_prep_epoch = 0;  // epochs (K0b: a new one; K4' prep: the next detect's)
  unsigned long long nf_force_epoch = 0;  // != 0: the epoch the next detects take (bsa_sim_detect_rows: the
                                         // records of every tile, prepared first, carry it)
  DevBuf sim_ctl;  // [0,24) gate {abort / non-finite, P, HK prediction}; [24,28) sticky abort; [32,40) steps
                   // done; [40,48) resopairs demand on a bookkeeping overflow; [48,56) pair-key
                   // block demand (several ranks); [56,64) an HK-kept list went stale in the batch
  // ASAS bookkeeping (bsa_asas.hip, resume_nav = 1): resopairs CSR over own
  // rows (+ next), per-row kept counts, LoS row pointers of the last call,
  // previous call's conflict / LoS CSR (one rank), stats
  DevBuf bk_rptr, bk_rcol, bk_nptr, bk_ncol, bk_cnt, bk_lptr, bk_pcptr, bk_plptr, bk_pccol, bk_plcol;
  DevBuf bk_stats, bk_tmp;
  unsigned long long bk_cap = 0;  // resopairs capacity (pairs)
  // several ranks: this rank's pair-key block and all ranks' blocks (this / the
  // previous call), bk_kw words per rank (grown on demand, the step retried)
  DevBuf bk_ksend, bk_kcur, bk_kprev;
  unsigned long long bk_kw = 0, bk_kw_alloc = 0;
  bool bk_ready = false;

  // halo exchange of the row-sharded resident step (bsa_halo.hip): each rank
  // receives only the column tiles its rows' boxes can reach (plus the tiles
  // of its resopairs' intruders) and prepares only those and its own tiles
  int halo_mode = 0;               // detect_enqueue (home mode): 0 off, 1 exchange (several ranks),
                                   // 2 one-GPU probe of one rank's share (bsa_sim_detect_rows)
  std::vector<int64_t> halo_cap;   // R x R tile capacities [sender * R + receiver], equal on all ranks
  DevBuf h_blk, h_gblk, h_plan, h_lists, h_send, h_recv, h_hl, h_dem;
  DevBuf h_present;                // plan reuse: the kept plan's present mask (k_halo_lists at a rebuild)
  int64_t halo_hl = 0;             // slots of the flat halo tile list (this rank's receive capacities)
  int64_t halo_grows = 0;          // capacity regrowths (aborted steps)
  int64_t halo_rx = 0, halo_tx = 0;  // bytes received / sent per CD step (the capacities' transfers)
  int halo_fields = 8;             // fp64 arrays per halo row of the last exchange (6 when derivable)
  bool last_fused = false;  // the last detect ran K1b fused into the prefilter (ExactFuse, bsa_cd.hip)
  bool fuse_skip = false;   // a fused detect ran out of flush records: its retry runs K1b as its own launch
  bool fuse_on = true;      // bsa_set_exact_fusion
  int fuse_recs = kFuseRecsMax;  // ... per-wave mid-sweep flush records (testing knob)
  int64_t fuse_count = 0, fuse_retries = 0;  // bsa_exact_fusion_stats
  // region layout agreement (comm_halo): every rank's send lengths / offsets
  // are compared with every receiver's expectation whenever the layout may have
  // changed -- a new capacity generation (init, regrowth: collective events) or
  // field count -- before any grouped send / recv is enqueued
  int64_t halo_cap_gen = 0, halo_chk_gen = -1;
  int halo_chk_nf = -1;
  int halo_tot_word = 0;           // h_dem word holding the last plan's received-tile total

  // 2-D wind field (bsa_set_windfield): lat lon vnorth veast of wf_nvec points
  DevBuf wfield;
  int64_t wf_nvec = 0;

  // resident step: per-pair MVP vectors evaluated inside K2 (k_rank) when set
  // (sim_cd sets it around detect_enqueue; full-N device arrays)
  const bsa_mvp_params *fuse_mvp = nullptr;
  const double *fuse_gse = nullptr, *fuse_gsn = nullptr, *fuse_vs = nullptr, *fuse_alt = nullptr;
  bool fuse_done = false;  // the last detect_enqueue produced the per-pair vectors
  bool fuse_rowdv = false;  // ... and folded them per row (k_rank_rows: mvp_rowdv)

  // standalone geo matrices (bsa_geo.hip)
  DevBuf geo_in, geo_pts, geo_out;
  hipEvent_t geo_ev[2] = {nullptr, nullptr};
  double geo_ms = 0.0;

  // ACDATA feed of the resident sim (bsa_feed.hip): pre-step altitude of the
  // last step (for traf.cas), device staging, pinned host mirror, completion event
  DevBuf s_altprev, feed_dev;
  // OpenAP flight envelope of the resident sim (bsa_sim_set_limits) + traf.ax
  DevBuf s_env, s_ax;
  bool sim_limits = false;
  // OpenAP flight-phase envelope (bsa_sim_set_perf): type table, per-aircraft
  // type index (int32) and the phase of the last step (u8)
  DevBuf s_ptab, s_ptype, s_phase;
  bool sim_perf = false;
  // NORESO / RESOOFF membership (bsa_sim_set_reso_lists, u8 in home order) and
  // the rows whose ResumeNav dropped a pair in the last CD call (u8, home order)
  DevBuf s_noreso, s_resooff, s_dropped;
  DevBuf s_atm;          // traf.p / rho / Temp = vatmos(traf.alt) of the last step (3 x n), when on
  bool sim_atmos = false;
  bool sim_noreso = false, sim_resooff = false;
  const uint8_t *fuse_noreso = nullptr;  // NORESO list for K2's fused MVP per-pair vectors
  int64_t sim_ntypes = 0;
  void *feed_host = nullptr;
  size_t feed_host_bytes = 0;
  hipEvent_t feed_ev = nullptr;
  bool feed_pending = false;
  int64_t feed_steps = 0, feed_rb = 0, feed_re = 0;
};

// device pointers for the MVP kernel (full-N traffic arrays, per-row outputs)
struct MvpDev {
  const double *gseast, *gsnorth, *vs, *alt, *trk, *gs, *selalt, *apvs;
  const double *aptrk, *aptas, *apalt;  // resident step, CR OFF (DoNothing.py) only; else NULL
  const uint8_t *noreso, *resooff;
  double *asas_alt, *o_trk, *o_tas, *o_vs;
  float *o_asase, *o_asasn;
  double *o_tsolv;
};
struct MvpIn;
// defer != NULL (resident step): the per-row kernel is not launched; its
// arguments go to *defer for the fused MVP + pilot + kinematics kernel
int mvp_device(Ctx *c, const bsa_mvp_params &p, const MvpDev &d, const unsigned *seg,
               const unsigned long long *gate, unsigned *sticky, const uint8_t *inconf, uint8_t *active,
               bool resolve, bool pairs_done = false, MvpIn *defer = nullptr);

// device pointers for the fused kinematics kernel
struct KinDev {
  const double *ptas, *phdg, *palt, *pvs, *bank, *eps, *accel;
  double *tas, *hdg, *alt, *vs, *lat, *lon;
  double *ax, *delspd, *cas, *mach, *gsnorth, *gseast, *gs, *trk, *coslat, *az;
  uint8_t *swhdgsel, *swaltsel;
};
int kin_device(Ctx *c, int64_t n, double simdt, int winddim, double vn, double ve, const KinDev &d);
struct WindField;
WindField wind_field(const Ctx *c);  // device view of the context's 2-D field (bsa_kin.hip)

// ASAS bookkeeping of one CD call (bsa_asas.hip): bk_count before the gate
// all-reduce and MVP (may raise the gate's bit 1 on resopairs overflow),
// bk_apply after MVP.  State arrays are full-N device arrays.
struct BkDev {
  const double *lat, *lon, *gse, *gsn, *trk;  // home order
  const unsigned *h2id, *id2h;                // home <-> aircraft index
  uint8_t *active;
  uint8_t *dropped;             // per row: ResumeNav dropped one of its pairs (waypoint recovery)
  unsigned long long *gate;
  unsigned *sticky;
  unsigned long long *demand;   // resopairs overflow: pairs needed
  unsigned long long *kdemand;  // several ranks, key block overflow: words needed
};
int bk_count(Ctx *c, const BkDev &d);
int bk_apply(Ctx *c, const BkDev &d);
void bk_release(Ctx *c);

// halo exchange (bsa_halo.hip; halo_pre / halo_mid and the device pieces in
// bsa_halo.h).  halo_mid: after K0 prepared the rank's own column tiles (and
// their boxes), plan which tiles every rank needs, exchange them (mode 1) and
// leave the flat list of this rank's halo tiles in h_hl (halo_hl slots, -1 =
// unused) and its present mask in h_plan
bool home_records(const Ctx *c, int64_t nrows);   // home-mode detect (of nrows rows) stores fp64 column records
int stage1_mid(int flags, bool reuse, int kwik);  // midpoint stage 1 for this detect?
int halo_init_caps(Ctx *c);      // bsa_sim_init, several ranks: exact initial capacities (no exchange)
int halo_grow(Ctx *c);           // after an aborted step, several ranks (collective)
void halo_release(Ctx *c);
const uint8_t *halo_present(const Ctx *c);  // the received-tile mask of the last halo_mid
const unsigned *halo_list_count(const Ctx *c);  // the probe's halo list length (device), else NULL
// K0b over every column tile (fused boxes, no per-detect zeroing): the halo
// plan's view of all tile boxes when every rank's state is on this GPU (bsa_cd.hip)
// every column tile's records and boxes (one K0b); nf_epoch != 0: non-finite
// columns store it into Ctx::nonfin (the detect that takes that epoch sees them)
int prep_all_tiles(Ctx *c, double rpz, double hpz, double tla, unsigned long long nf_epoch = 0);

// exclusive prefix sum of n words, one launch (bsa_cd.hip)
int scan_excl(Ctx *c, const unsigned *in, unsigned *out, int n);
// spatial (home) order of the n aircraft in own[] (bsa_cd.hip): home -> aircraft index
int home_order(Ctx *c, double tla, std::vector<unsigned> &h2id);
// the last detect's pair lists and per-row outputs in aircraft-index terms
// (bsa_ctx.hip): home rows -> indices, rows in ascending index order
struct HostPairs {
  std::vector<int32_t> ci, cj, li, lj;
  std::vector<double> pay;  // 5 x P (qdr dist tcpa tinconf dcpa)
  std::vector<uint8_t> inconf;
  std::vector<double> tcpamax;
};
int download_pairs(Ctx *c, HostPairs &h);
void home_pairs_to_ids(const Ctx *c, int64_t rb, HostPairs &h);
// resident sim (bsa_sim.hip): the maps of Ctx::h2id_h (host + device, lpos of this rank's rows)
int set_home_maps(Ctx *c);
// this rank's 512-aligned home range [sim_rb, sim_re) and rows per rank for c->n (bsa_sim.hip)
void set_rank_rows(Ctx *c);

// error helpers
int fail(Ctx *c, const char *fmt, ...);
#define BSA_HIP(c, call)                                                              \
  do {                                                                                \
    hipError_t e_ = (call);                                                           \
    if (e_ != hipSuccess)                                                             \
      return ::bsa::fail((c), "%s failed: %s (%s:%d)", #call, hipGetErrorString(e_), \
                         __FILE__, __LINE__);                                         \
  } while (0)

// collectives (bsa_comm.hip): RCCL or the in-process group, stream-ordered;
// no-ops (plain copies) with one rank
bool comm_multi(const Ctx *c);
int comm_allgather(Ctx *c, const void *send, void *recv, size_t bytes);  // recv: nranks x bytes
int comm_allreduce_max_u64(Ctx *c, unsigned long long *buf, int count); // device words, in place
int comm_allgather_inplace(Ctx *c, double *const *f, int nf, size_t rpr); // rank blocks of nf arrays
int comm_allreduce_host(Ctx *c, double *v, int count, bool max);         // host values (synchronises)
int comm_gatherv(Ctx *c, int root, const void *send, size_t bytes, void *recv, const size_t *off,
                 const size_t *len);                                     // rank-order blocks to root
int comm_halo(Ctx *c, const void *send, const size_t *soff, const size_t *slen, size_t stot, void *recv,
              const size_t *roff, const size_t *rlen, const size_t *peer);  // halo regions (bsa_halo.hip)
void comm_release(Ctx *c);

// sim / comm teardown (bsa_sim.hip); ACDATA feed teardown (bsa_feed.hip)
void sim_release(Ctx *c);
void feed_release(Ctx *c);
int sim_adopt_pairs(Ctx *c);  // after resident steps: the last CD call's pairs become fetchable

// detect entry points (bsa_cd.hip): detect = enqueue + finish (+ retries)
int detect(Ctx *c, double rpz, double hpz, double tla, int flags, int64_t rb, int64_t re,
           int64_t *n_conf, int64_t *n_los);
bool nonfin_word(Ctx *c);  // Ctx::nonfin allocated (zeroed when new)
int detect_enqueue(Ctx *c, double rpz, double hpz, double tla, int flags, int64_t rb, int64_t re,
                   unsigned long long *gate);
int detect_finish(Ctx *c, bool *retry);
#ifdef BSA_PF_TRACE
int pf_trace_dump(Ctx *c, unsigned long long groups, unsigned long long tiles);  // (diagnostic builds)
#endif
void grow_k2_bucket(Ctx *c, unsigned long long demand);

}  // namespace bsa
