// ACDATA feed of the GPU-resident sim: the per-aircraft
// stream ScreenIO.send_aircraft_data publishes at 5 Hz
// (bluesky/simulation/qtgl/screenio.py:194-239: lat lon alt tas cas gs trk vs,
// asas.inconf / tcpamax, the four pair counts, asasn / asase) served from the
// device without stalling the sim: bsa_sim_acdata_request enqueues one pack
// kernel + one D2H copy into a pinned host mirror behind the queued steps and
// records an event; bsa_sim_acdata_poll copies the mirror out once that event
// has completed (or waits for it).  No collective: each rank serves its own
// rows [row_begin, row_end), concatenated in rank order by the caller.
#include "bsa_internal.h"
#include "bsa_kin_math.h"

namespace bsa {

// Mirror layout (rows nr): 8 x u64 header | 9 x nr fp64 | 2 x nr f32 | nr u8
constexpr int kFeedF64 = 9;  // lat lon alt tas cas gs trk vs tcpamax

static size_t feed_bytes(int64_t nr) { return 64 + (size_t)nr * (kFeedF64 * 8 + 2 * 4 + 1); }

struct FeedSrc {
  const double *f[kFeedF64 - 1];        // lat lon alt tas [altprev] gs trk vs (full n, row k)
  int stepped;                          // a step ran: slot 4 holds the pre-step altitude
  const double *tcpamax;                // last CD call's rows (row k - rb), may be NULL
  const float *asasn, *asase;           // full n
  const uint8_t *inconf;                // last CD call's rows, may be NULL
  const unsigned long long *bk_stats;   // ASAS bookkeeping counters, may be NULL
};

__global__ __launch_bounds__(256) void k_feed_pack(int64_t rb, int64_t nr, FeedSrc s, char *__restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long *hdr = (unsigned long long *)out;
  if (r < 8) hdr[r] = (s.bk_stats && r >= 1 && r <= 4) ? s.bk_stats[r] : 0ull;
  if (r >= nr) return;
  double *f64 = (double *)(out + 64);
  const int64_t k = rb + r;
#pragma unroll
  for (int f = 0; f < kFeedF64 - 1; ++f) f64[f * nr + r] = s.f[f][k];
  // traf.cas = vtas2cas(tas, alt) in UpdateAirSpeed, i.e. with the step's new
  // tas and its pre-step altitude (traffic.py:434, before UpdatePosition)
  f64[4 * nr + r] = s.stepped ? kin::vtas2cas(s.f[3][k], s.f[4][k]) : 0.0;
  f64[(kFeedF64 - 1) * nr + r] = s.tcpamax ? s.tcpamax[r] : 0.0;
  float *f32 = (float *)(f64 + kFeedF64 * nr);
  f32[r] = s.asasn[k];
  f32[nr + r] = s.asase[k];
  uint8_t *u8 = (uint8_t *)(f32 + 2 * nr);
  u8[r] = s.inconf ? s.inconf[r] : 0;
}

void feed_release(Ctx *c) {
  if (c->feed_ev) (void)hipEventDestroy(c->feed_ev);
  c->feed_ev = nullptr;
  if (c->feed_host) (void)hipHostFree(c->feed_host);
  c->feed_host = nullptr;
  c->feed_host_bytes = 0;
  c->feed_pending = false;
  release(c->feed_dev);
}

static int feed_request(Ctx *c) {
  if (!c->sim_ready) return fail(c, "ACDATA request before bsa_sim_init");
  const int64_t rb = c->sim_rb, nr = c->sim_re - c->sim_rb;
  const size_t bytes = feed_bytes(nr);
  if (c->feed_pending) BSA_HIP(c, hipEventSynchronize(c->feed_ev));  // the mirror is about to be rewritten
  if (!ensure(c, c->feed_dev, bytes, "ACDATA staging")) return -1;
  if (c->feed_host_bytes < bytes) {
    if (c->feed_host) BSA_HIP(c, hipHostFree(c->feed_host));
    c->feed_host = nullptr;
    c->feed_host_bytes = 0;
    BSA_HIP(c, hipHostMalloc(&c->feed_host, bytes, hipHostMallocDefault));
    c->feed_host_bytes = bytes;
  }
  if (!c->feed_ev) BSA_HIP(c, hipEventCreateWithFlags(&c->feed_ev, hipEventDisableTiming));
  // inconf / tcpamax hold the last CD call's rows (the rank's rows once a CD step ran)
  const bool have_cd = c->sim_cd_calls > 0 && c->inconf.p && c->last_rb == rb && c->last_re == c->sim_re;
  FeedSrc s;
  const void *src[kFeedF64 - 1] = {c->own[0].p, c->own[1].p, c->own[4].p, c->s_tas.p,
                                   c->s_altprev.p, c->own[3].p, c->own[2].p, c->own[5].p};
  for (int f = 0; f < kFeedF64 - 1; ++f) s.f[f] = (const double *)src[f];
  s.stepped = c->sim_steps > 0;
  s.tcpamax = have_cd ? (const double *)c->tcpamax.p : nullptr;
  s.inconf = have_cd ? (const uint8_t *)c->inconf.p : nullptr;
  s.asasn = (const float *)c->s_asn.p;
  s.asase = (const float *)c->s_ase.p;
  s.bk_stats = (c->simp.resume_nav && c->bk_ready) ? (const unsigned long long *)c->bk_stats.p : nullptr;
  const int64_t threads = std::max<int64_t>(nr, 8);
  k_feed_pack<<<(unsigned)((threads + 255) / 256), 256, 0, c->stream>>>(rb, nr, s, (char *)c->feed_dev.p);
  BSA_HIP(c, hipGetLastError());
  BSA_HIP(c, hipMemcpyAsync(c->feed_host, c->feed_dev.p, bytes, hipMemcpyDeviceToHost, c->stream));
  BSA_HIP(c, hipEventRecord(c->feed_ev, c->stream));
  c->feed_pending = true;
  c->feed_steps = c->sim_steps;
  c->feed_rb = rb;
  c->feed_re = c->sim_re;
  return 0;
}

static int feed_poll(Ctx *c, int wait, bsa_acdata *o) {
  if (!c->feed_pending) return fail(c, "no ACDATA snapshot requested");
  if (wait) {
    BSA_HIP(c, hipEventSynchronize(c->feed_ev));
  } else {
    const hipError_t e = hipEventQuery(c->feed_ev);
    if (e == hipErrorNotReady) return 1;
    if (e != hipSuccess) return fail(c, "hipEventQuery: %s", hipGetErrorString(e));
  }
  const int64_t nr = c->feed_re - c->feed_rb;
  const unsigned long long *hdr = (const unsigned long long *)c->feed_host;
  const bool counts = c->simp.resume_nav != 0;  // global counts, the same on every rank
  o->steps = c->feed_steps;
  o->row_begin = c->feed_rb;
  o->row_end = c->feed_re;
  o->nconf_cur = counts ? (int64_t)hdr[1] : -1;
  o->nlos_cur = counts ? (int64_t)hdr[2] : -1;
  o->nconf_tot = counts ? (int64_t)hdr[3] : -1;
  o->nlos_tot = counts ? (int64_t)hdr[4] : -1;
  // the mirror holds the rows in home order: row r goes to lpos[r], its place
  // among the rank's rows in ascending aircraft index (all aircraft with one rank)
  const unsigned *L = c->lpos_h.data();
  auto put = [&](auto *dst, const auto *src) {
    if (dst)
      for (int64_t r = 0; r < nr; ++r) dst[L[r]] = src[r];
  };
  const double *f64 = (const double *)((const char *)c->feed_host + 64);
  double *dst[kFeedF64] = {o->lat, o->lon, o->alt, o->tas, o->cas, o->gs, o->trk, o->vs, o->tcpamax};
  for (int f = 0; f < kFeedF64; ++f) put(dst[f], f64 + f * nr);
  const float *f32 = (const float *)(f64 + kFeedF64 * nr);
  put(o->asasn, f32);
  put(o->asase, f32 + nr);
  put(o->inconf, (const uint8_t *)(f32 + 2 * nr));
  return 0;
}

}  // namespace bsa

extern "C" {

int bsa_sim_acdata_request(bsa_ctx *cc) {
  bsa::Ctx *c = (bsa::Ctx *)cc;
  if (!c) return -1;
  BSA_HIP(c, hipSetDevice(c->device));
  return bsa::feed_request(c);
}

int bsa_sim_acdata_poll(bsa_ctx *cc, int wait, bsa_acdata *out) {
  bsa::Ctx *c = (bsa::Ctx *)cc;
  if (!c) return -1;
  if (!out) return bsa::fail(c, "NULL bsa_acdata");
  BSA_HIP(c, hipSetDevice(c->device));
  return bsa::feed_poll(c, wait, out);
}

}  // extern "C"
