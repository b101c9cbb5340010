// Device restatements of bluesky/tools/geo.py shared by the fused CD kernel
// (bsa_cd.hip, K1b) and the standalone matrix producers (bsa_geo.hip).
// Same operation order as the numpy code, compiled with -ffp-contract=off,
// so every + - * / sqrt rounds like numpy's.
#pragma once
#include "bsa_internal.h"

#pragma clang fp contract(off)

namespace bsa {

// numpy.maximum / numpy.minimum semantics: NaN propagates, ties keep `a`.
__device__ __forceinline__ double np_max(double a, double b) {
  return (a >= b || a != a) ? a : b;
}
__device__ __forceinline__ double np_min(double a, double b) {
  return (a <= b || a != a) ? a : b;
}

// fmod(a, 360) without the library's loop, exactly fmod's value: for
// 360 <= |a| < 360 2^30, q = trunc(|a| (1/360)) is the true quotient or one
// off (the product's error is < 2^-22 of one: two roundings of 2^-53 relative
// on a quotient below 2^30; no division needed), q 360 is exact (9
// significant bits times < 2^30) and |a| - q 360 is exact by Sterbenz (|a| in
// [q 360 / 2, 2 q 360] for the true q and its neighbours that are tried, q = 0
// only for |a| < 720), so the remainder of the true quotient comes out
// exactly; fmod's sign is a's.  Anything else (huge, inf, NaN) goes to fmod.
__device__ __forceinline__ double fmod360(double a) {
  const double aa = fabs(a);
  if (aa < 360.0) return a;
  if (!(aa < 386547056640.0)) return fmod(a, 360.0);  // 360 * 2^30
  double q = trunc(aa * (1.0 / 360.0));
  double r = aa - q * 360.0;
  if (r < 0.0) {
    q -= 1.0;
    r = aa - q * 360.0;
  } else if (r >= 360.0) {
    q += 1.0;
    r = aa - q * 360.0;
  }
  return copysign(r, a);
}

// numpy.remainder for float64 (npy_divmod semantics), b > 0.  fmod is exact
// and returns a itself when |a| < b, so that common case skips fmod's loop
// (and b = 360 takes fmod360).
__device__ __forceinline__ double np_rem(double a, double b) {
  double mod = (fabs(a) < b) ? a : (b == 360.0 ? fmod360(a) : fmod(a, b));
  if (mod != 0.0) {
    if ((b < 0) != (mod < 0)) mod += b;
  } else {
    mod = copysign(0.0, b);
  }
  return mod;
}

// geo.py:32-54 rwgs84_matrix, elementwise, same op order.
// rwgs84_sc: the same from sin / cos(radians(latd)) a caller already holds
__device__ __forceinline__ double rwgs84_sc(double sinlat, double coslat) {
  const double a = kWGS84_A, b = kWGS84_B;
  const double an = (a * a) * coslat;
  const double bn = (b * b) * sinlat;
  const double ad = a * coslat;
  const double bd = b * sinlat;
  const double anan = an * an;
  const double bnbn = bn * bn;
  const double adad = ad * ad;
  const double bdbd = bd * bd;
  return sqrt((anan + bnbn) / (adad + bdbd));
}
// sin and cos of one argument: one sincos (SC; bit for bit the separate
// calls, tools/sincos_check.hip), or the separate calls -- for the fused
// prefilter's K1b, where sincos's result pointers raised the kernel's
// register pressure (scratch 24 -> 56 B per lane, +8 MB of spill writes per
// launch at the 100k box)
template <bool SC>
__device__ __forceinline__ void sin_cos(double x, double *s, double *c) {
  if (SC) {
    sincos(x, s, c);
  } else {
    *s = sin(x);
    *c = cos(x);
  }
}
template <bool SC = true>
__device__ __forceinline__ double rwgs84(double latd) {
  double sinlat, coslat;
  sin_cos<SC>(latd * kD2R, &sinlat, &coslat);
  return rwgs84_sc(sinlat, coslat);
}

// Per-point factors of qdrdist_matrix's broadcasts (geo.py:127,136-140).
struct GeoPt {
  double lat, lon, sinlat, coslat;
  double hemA;  // |lat| * (rwgs84(lat) + a)      geo.py:127
};
__device__ __forceinline__ GeoPt geo_pt(double lat, double lon) {
  GeoPt p;
  p.lat = lat;
  p.lon = lon;
  sincos(lat * kD2R, &p.sinlat, &p.coslat);
  p.hemA = fabs(lat) * (rwgs84_sc(p.sinlat, p.coslat) + kWGS84_A);
  return p;
}

// One entry [i, j] of geo.qdrdist_matrix (geo.py:117-160): point 1 = row i,
// point 2 = column j, eps = (lat1[j] == 0.) * 1e-6 (geo.py:128, indexed by
// the column).  qdr [deg], dist [nm].
template <bool SC = true>
__device__ __forceinline__ void qdrdist_entry(double lat1, double lon1, double sinlat1, double coslat1,
                                              double hemA1, double lat2, double lon2, double sinlat2,
                                              double coslat2, double hemA2, double eps, double &qdr,
                                              double &dist_nm) {
  const double prodla = lat1 * lat2;
  double rr;
  if (prodla < 0) {
    // different hemisphere (geo.py:125-128)
    rr = (0.5 * (hemA1 + hemA2)) / (fabs(lat1) + (fabs(lat2) + eps));
  } else {
    rr = rwgs84<SC>(lat1 + lat2);  // geo.py:121: radius at the SUM of the latitudes
  }
  const double sin1 = (lat2 - lat1) * kD2R;
  const double sin2 = (lon2 - lon1) * kD2R;
  double sin21, cos21;
  sin_cos<SC>(sin2, &sin21, &cos21);
  const double y = sin21 * coslat2;
  const double x1 = coslat1 * sinlat2;
  const double x2 = sinlat1 * coslat2;
  const double x3 = x2 * cos21;
  const double x = x1 - x3;
  qdr = atan2(y, x) * kR2D;
  const double sin10 = fabs(sin(sin1 / 2.));
  const double sin20 = fabs(sin(sin2 / 2.));
  const double sin1sin1 = sin10 * sin10;
  const double sin2sin2 = sin20 * sin20;
  const double hav = sin1sin1 + (coslat1 * coslat2) * sin2sin2;
  const double dist_c = 2. * atan2(sqrt(hav), sqrt(1 - hav));
  dist_nm = (rr / kNM) * dist_c;
}

// One entry [i, j] of geo.kwikqdrdist_matrix (geo.py:351-361):
// dlat = latb[j] - lata[i], dlon = lonb[j] - lona[i], and the caller passes
// cavelat's latitudes as written, lata[j] + latb[i] (geo.py:355).
// qdr [deg] in [0, 360), dist [m].
__device__ __forceinline__ void kwik_entry(double lata_i, double lona_i, double latb_j, double lonb_j,
                                           double cavesum, double &qdr, double &dist_m) {
  const double dlat = (latb_j - lata_i) * kD2R;
  const double dlon = (lonb_j - lona_i) * kD2R;
  const double cavelat = cos((cavesum * kD2R) * 0.5);
  const double dangle = sqrt(dlat * dlat + (dlon * dlon) * (cavelat * cavelat));
  dist_m = 6371000. * dangle;
  qdr = np_rem(atan2(dlon * cavelat, dlat) * kR2D, 360.);
}

}  // namespace bsa
