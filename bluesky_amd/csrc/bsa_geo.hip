// Standalone materialised geo matrices (include/bsaccel.h "geo matrices"):
//   geo.qdrdist_matrix      bluesky/tools/geo.py:110-162
//   geo.kwikqdrdist_matrix  bluesky/tools/geo.py:347-363
// as the reference's callers outside the CD use them (traffic/metric.py:596,
// 711,1188: 1 x m and 1 x n np.matrix operands -> m x n outer matrices;
// traffic/asas/SSD.py:169: 1-D operands -> element-wise pairs).
//
// The outer producers write 16 B per entry (qdr + dist, fp64) and read only
// two cached point vectors, so they are HBM-write-bound once the fp64 libm
// work per entry (qdrdist: 6 sin/cos/atan2 + rwgs84's sin/cos/sqrt; KWIK: cos,
// atan2, fmod) keeps up: one workgroup per (row, 2048-column chunk), every
// lane owns 8 columns 256 apart (coalesced non-temporal stores, the row's
// factors in registers, the column factors from L2).
#include "bsa_geo_math.h"
#include "bsa_internal.h"

#pragma clang fp contract(off)

namespace bsa {

constexpr int kGeoThreads = 256;
constexpr int kGeoPerLane = 8;
constexpr int kGeoChunk = kGeoThreads * kGeoPerLane;  // columns per workgroup

__global__ __launch_bounds__(256) void k_geo_pts(int64_t n, const double *__restrict__ lat,
                                                 const double *__restrict__ lon, GeoPt *__restrict__ out) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) out[k] = geo_pt(lat[k], lon[k]);
}

__device__ __forceinline__ void store_nt(double *p, double v) { __builtin_nontemporal_store(v, p); }

// qdrdist_matrix, outer: out[i*n + j].  eps of column j = (lat1[j] == 0)*1e-6
// (geo.py:128); with m == 1 lat1 has one element, broadcast over the columns.
__global__ __launch_bounds__(256) void k_qdrdist_outer(int64_t m, int64_t n, int64_t nchunk,
                                                       const GeoPt *__restrict__ p1,
                                                       const GeoPt *__restrict__ p2,
                                                       const double *__restrict__ lat1,
                                                       double *__restrict__ qdr, double *__restrict__ dist) {
  const int64_t i = (int64_t)blockIdx.x / nchunk;
  const int64_t j0 = ((int64_t)blockIdx.x - i * nchunk) * kGeoChunk + threadIdx.x;
  const GeoPt a = p1[i];
  const double eps_all = (m == 1) ? ((lat1[0] == 0.0) ? 0.000001 : 0.0) : 0.0;
#pragma unroll
  for (int e = 0; e < kGeoPerLane; ++e) {
    const int64_t j = j0 + (int64_t)e * kGeoThreads;
    if (j >= n) break;
    const GeoPt b = p2[j];
    const double eps = (m == 1) ? eps_all : ((lat1[j] == 0.0) ? 0.000001 : 0.0);
    double q, d;
    qdrdist_entry(a.lat, a.lon, a.sinlat, a.coslat, a.hemA, b.lat, b.lon, b.sinlat, b.coslat, b.hemA, eps,
                  q, d);
    const int64_t o = i * n + j;
    if (qdr) store_nt(qdr + o, q);
    if (dist) store_nt(dist + o, d);
  }
}

// kwikqdrdist_matrix, outer (m == n): out[i*n + j], cavelat at lata[j] + latb[i].
__global__ __launch_bounds__(256) void k_kwik_outer(int64_t n, int64_t nchunk, const double *__restrict__ lata,
                                                    const double *__restrict__ lona,
                                                    const double *__restrict__ latb,
                                                    const double *__restrict__ lonb,
                                                    double *__restrict__ qdr, double *__restrict__ dist) {
  const int64_t i = (int64_t)blockIdx.x / nchunk;
  const int64_t j0 = ((int64_t)blockIdx.x - i * nchunk) * kGeoChunk + threadIdx.x;
  const double la = lata[i], lo = lona[i], lbi = latb[i];
#pragma unroll
  for (int e = 0; e < kGeoPerLane; ++e) {
    const int64_t j = j0 + (int64_t)e * kGeoThreads;
    if (j >= n) break;
    double q, d;
    kwik_entry(la, lo, latb[j], lonb[j], lata[j] + lbi, q, d);
    const int64_t o = i * n + j;
    if (qdr) store_nt(qdr + o, q);
    if (dist) store_nt(dist + o, d);
  }
}

// element-wise pairs (1-D operands, SSD.py:169): every product is per k
__global__ __launch_bounds__(256) void k_geo_pairwise(int64_t m, int kwik, const double *__restrict__ lat1,
                                                      const double *__restrict__ lon1,
                                                      const double *__restrict__ lat2,
                                                      const double *__restrict__ lon2,
                                                      double *__restrict__ qdr, double *__restrict__ dist) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= m) return;
  double q, d;
  if (kwik) {
    kwik_entry(lat1[k], lon1[k], lat2[k], lon2[k], lat1[k] + lat2[k], q, d);
  } else {
    const GeoPt a = geo_pt(lat1[k], lon1[k]);
    const GeoPt b = geo_pt(lat2[k], lon2[k]);
    qdrdist_entry(a.lat, a.lon, a.sinlat, a.coslat, a.hemA, b.lat, b.lon, b.sinlat, b.coslat, b.hemA,
                  (lat1[k] == 0.0) ? 0.000001 : 0.0, q, d);
  }
  if (qdr) store_nt(qdr + k, q);
  if (dist) store_nt(dist + k, d);
}

static int geo_run(Ctx *c, int64_t m, const double *lat1, const double *lon1, int64_t n, const double *lat2,
                   const double *lon2, int flags, double *qdr, double *dist) {
  const bool kwik = flags & BSA_GEO_KWIK, pairwise = flags & BSA_GEO_PAIRWISE;
  if (flags & ~(BSA_GEO_KWIK | BSA_GEO_PAIRWISE)) return fail(c, "unknown geo flags 0x%x", flags);
  if (m < 0 || n < 0) return fail(c, "negative size");
  if (!lat1 || !lon1 || !lat2 || !lon2) return fail(c, "NULL input array");
  if (pairwise && m != n)
    return fail(c, "pairwise operands must have equal length (m=%lld, n=%lld)", (long long)m, (long long)n);
  if (!pairwise && kwik && m != n)
    return fail(c, "kwikqdrdist_matrix outer form needs m == n (cavelat is indexed [j, i], geo.py:355); "
                   "m=%lld, n=%lld", (long long)m, (long long)n);
  if (!pairwise && !kwik && m != n && m != 1)
    return fail(c, "qdrdist_matrix outer form needs m == n or m == 1 ((lat1 == 0.)*1e-6 is added to the "
                   "n-vector lat2, geo.py:128); m=%lld, n=%lld", (long long)m, (long long)n);
  const int64_t total = pairwise ? m : m * n;
  c->geo_ms = 0.0;
  if (total == 0) return 0;
  if (!ensure(c, c->geo_in, (size_t)(2 * m + 2 * n) * 8, "geo inputs")) return -1;
  if (!ensure(c, c->geo_out, (size_t)total * 16, "geo outputs")) return -1;
  double *d_lat1 = (double *)c->geo_in.p, *d_lon1 = d_lat1 + m, *d_lat2 = d_lon1 + m, *d_lon2 = d_lat2 + n;
  double *d_qdr = qdr ? (double *)c->geo_out.p : nullptr;
  double *d_dist = dist ? (double *)c->geo_out.p + total : nullptr;
  BSA_HIP(c, hipMemcpyAsync(d_lat1, lat1, m * 8, hipMemcpyHostToDevice, c->stream));
  BSA_HIP(c, hipMemcpyAsync(d_lon1, lon1, m * 8, hipMemcpyHostToDevice, c->stream));
  BSA_HIP(c, hipMemcpyAsync(d_lat2, lat2, n * 8, hipMemcpyHostToDevice, c->stream));
  BSA_HIP(c, hipMemcpyAsync(d_lon2, lon2, n * 8, hipMemcpyHostToDevice, c->stream));
  for (int k = 0; k < 2; ++k)
    if (!c->geo_ev[k]) BSA_HIP(c, hipEventCreateWithFlags(&c->geo_ev[k], hipEventDisableSystemFence));
  GeoPt *p1 = nullptr, *p2 = nullptr;
  if (!pairwise && !kwik) {
    if (!ensure(c, c->geo_pts, (size_t)(m + n) * sizeof(GeoPt), "geo points")) return -1;
    p1 = (GeoPt *)c->geo_pts.p;
    p2 = p1 + m;
    k_geo_pts<<<(unsigned)((m + 255) / 256), 256, 0, c->stream>>>(m, d_lat1, d_lon1, p1);
    k_geo_pts<<<(unsigned)((n + 255) / 256), 256, 0, c->stream>>>(n, d_lat2, d_lon2, p2);
  }
  BSA_HIP(c, hipEventRecord(c->geo_ev[0], c->stream));
  if (pairwise) {
    k_geo_pairwise<<<(unsigned)((m + 255) / 256), 256, 0, c->stream>>>(m, kwik ? 1 : 0, d_lat1, d_lon1, d_lat2,
                                                                       d_lon2, d_qdr, d_dist);
  } else {
    const int64_t nchunk = (n + kGeoChunk - 1) / kGeoChunk;
    const int64_t blocks = m * nchunk;
    if (blocks > 0x7fffffffLL) return fail(c, "geo matrix too large for one launch (%lld x %lld)",
                                           (long long)m, (long long)n);
    if (kwik)
      k_kwik_outer<<<(unsigned)blocks, kGeoThreads, 0, c->stream>>>(n, nchunk, d_lat1, d_lon1, d_lat2, d_lon2,
                                                                    d_qdr, d_dist);
    else
      k_qdrdist_outer<<<(unsigned)blocks, kGeoThreads, 0, c->stream>>>(m, n, nchunk, p1, p2, d_lat1, d_qdr,
                                                                       d_dist);
  }
  BSA_HIP(c, hipGetLastError());
  BSA_HIP(c, hipEventRecord(c->geo_ev[1], c->stream));
  if (qdr) BSA_HIP(c, hipMemcpyAsync(qdr, d_qdr, total * 8, hipMemcpyDeviceToHost, c->stream));
  if (dist) BSA_HIP(c, hipMemcpyAsync(dist, d_dist, total * 8, hipMemcpyDeviceToHost, c->stream));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  float ms = 0.f;
  BSA_HIP(c, hipEventElapsedTime(&ms, c->geo_ev[0], c->geo_ev[1]));
  c->geo_ms = ms;
  return 0;
}

}  // namespace bsa

extern "C" {

int bsa_qdrdist(bsa_ctx *cc, int64_t m, const double *lat1, const double *lon1, int64_t n, const double *lat2,
                const double *lon2, int flags, double *qdr, double *dist) {
  bsa::Ctx *c = (bsa::Ctx *)cc;
  if (!c) return -1;
  BSA_HIP(c, hipSetDevice(c->device));
  return bsa::geo_run(c, m, lat1, lon1, n, lat2, lon2, flags, qdr, dist);
}

int bsa_geo_last_ms(bsa_ctx *cc, double *ms) {
  bsa::Ctx *c = (bsa::Ctx *)cc;
  if (!c || !ms) return -1;
  *ms = c->geo_ms;
  return 0;
}

}  // extern "C"
