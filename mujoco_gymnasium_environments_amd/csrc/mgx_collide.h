// mgx_collide.h — narrowphase primitives, one candidate pair per lane.
//
// Semantics follow MuJoCo's mjc_* collision functions [ext] (reached from mj_collision in
// mj_step, humanoid_soccer_env/soccer_env.py:414): geom types ordered type1 <= type2, contact
// normal points from geom1 to geom2, `dist` is the signed surface distance (negative =
// penetration), `pos` is the midpoint between the two surfaces, and a contact exists when
// dist <= margin. Sphere-capsule and capsule-capsule restate mjc_SphereCapsule /
// mjc_CapsuleCapsule (centre + half-axis form, parallel axes up to two contacts); capsule-box
// follows mjc_CapsuleBox's structure (closest / deepest axis point as a sphere-box contact, a
// second one along a face, <= 2); box-box uses separating axes + reference/incident face clipping
// (<= 8 contacts, own design). The CPU oracle (oracle/mjref.c) restates the same algorithms in fp64.
#pragma once
#include "mgx_common.h"

namespace mgx {

template <typename T>
struct Con { T dist, pos[3], n[3]; };

template <typename T>
__device__ __forceinline__ void seg_ends(const T* pos, const T* mat, T hl, T* a, T* b) {
  for (int k = 0; k < 3; k++) { a[k] = pos[k] - hl * mat[3 * k + 2]; b[k] = pos[k] + hl * mat[3 * k + 2]; }
}

template <typename T>
__device__ __forceinline__ void seg_seg(const T* p1, const T* q1, const T* p2, const T* q2, T* s, T* t) {
  T d1[3], d2[3], r[3];
  for (int k = 0; k < 3; k++) { d1[k] = q1[k] - p1[k]; d2[k] = q2[k] - p2[k]; r[k] = p1[k] - p2[k]; }
  T a = dot3(d1, d1), e = dot3(d2, d2), f = dot3(d2, r);
  if (a <= minval<T>() && e <= minval<T>()) { *s = *t = 0; return; }
  if (a <= minval<T>()) { *s = 0; *t = clampv(f / e, (T)0, (T)1); return; }
  T c = dot3(d1, r);
  if (e <= minval<T>()) { *t = 0; *s = clampv(-c / a, (T)0, (T)1); return; }
  T b = dot3(d1, d2), den = a * e - b * b;
  T ss = den > (T)1e-12 * a * e ? clampv((b * f - c * e) / den, (T)0, (T)1) : (T)0;
  T tt = (b * ss + f) / e;
  if (tt < 0) { tt = 0; ss = clampv(-c / a, (T)0, (T)1); }
  else if (tt > 1) { tt = 1; ss = clampv((b - c) / a, (T)0, (T)1); }
  *s = ss; *t = tt;
}

template <typename T>
__device__ __forceinline__ T box_sd(const T* p, const T* h, T* e) {
  // a coordinate within `tie` outside its face plane counts as on it: points placed on a face's
  // boundary by construction (capsule_box) classify the same under any rounding
  const T tie = (sizeof(T) == 8 ? (T)1e-12 : (T)1e-6) * (h[0] + h[1] + h[2]);
  bool outside = false;
  T dv[3];
  for (int k = 0; k < 3; k++) {
    T q = clampv(p[k], -h[k], h[k]);
    dv[k] = p[k] - q;
    if (fabs(dv[k]) <= tie) dv[k] = 0;
    if (dv[k] != 0) outside = true;
  }
  if (outside) {
    T L = normalize3(dv);
    e[0] = dv[0]; e[1] = dv[1]; e[2] = dv[2];
    return L;
  }
  // nearest face; faces within `tie` of the nearest count as equally near and the lowest axis
  // wins, so two implementations with different rounding pick the same face at a kink (the
  // deepest point of a capsule axis inside a box is where two face distances are equal)
  int best = 0;
  T bd = h[0] - fabs(p[0]);
  for (int k = 1; k < 3; k++) {
    T dk = h[k] - fabs(p[k]);
    if (dk < bd - tie) { bd = dk; best = k; }
  }
  e[0] = e[1] = e[2] = 0;
  e[best] = p[best] >= -tie ? (T)1 : (T)-1;  // on the mid-plane (within tie) the + face
  return -bd;
}

template <typename T>
__device__ __forceinline__ int sphere_box_core(const T* c, T r, const T* bp, const T* bm, const T* h, T margin, Con<T>* out) {
  T tmp[3] = {c[0] - bp[0], c[1] - bp[1], c[2] - bp[2]}, pl[3], e[3], ew[3];
  mulmatTvec3(pl, bm, tmp);
  T sd = box_sd(pl, h, e);
  T dist = sd - r;
  if (dist > margin) return 0;
  mulmatvec3(ew, bm, e);
  out->dist = dist;
  for (int k = 0; k < 3; k++) { out->n[k] = -ew[k]; out->pos[k] = c[k] - ew[k] * (r + (T)0.5 * dist); }
  return 1;
}

// Point of a capsule axis closest to (outside) or deepest in (inside) a box, in the box frame:
// the axis is c + s a, s in [-1, 1]. The signed distance d(s) of the point to the box is convex
// and piecewise smooth, so its minimum over [-1, 1] lies at an end, a kink or a stationary point
// of a piece: the 2 ends, where a coordinate crosses a face plane (6) or zero (3), where two
// inside face distances are equal (12), and the stationary point of every outside piece (26
// sign patterns). All 49 candidates are evaluated exactly (generated on the fly, twice: no
// per-lane arrays); the lowest s within tol of the minimum wins, so an axis lying flat on a face
// starts at the end of its overlap with the face. The result depends only on the candidate set.
template <typename T>
__device__ __forceinline__ bool capsule_box_cand(int k, const T* c, const T* a, const T* h, T& s) {
  if (k < 2) { s = k ? (T)1 : (T)-1; return true; }
  if (k < 11) {
    const int i = (k - 2) / 3, r = (k - 2) % 3;
    if (!(fabs(a[i]) > minval<T>())) return false;
    s = (r == 0 ? h[i] - c[i] : r == 1 ? -h[i] - c[i] : -c[i]) / a[i];
    return true;
  }
  if (k < 23) {
    const int q = (k - 11) >> 2, sg = (k - 11) & 3;
    const int i = q == 2 ? 1 : 0, j = q == 0 ? 1 : 2;
    const T si = (sg & 1) ? (T)-1 : (T)1, sj = (sg & 2) ? (T)-1 : (T)1;
    const T den = sj * a[j] - si * a[i];
    if (!(fabs(den) > minval<T>())) return false;
    s = (h[j] - h[i] - sj * c[j] + si * c[i]) / den;
    return true;
  }
  int q = k - 22;  // sign pattern 1..26: per axis 0 inside, 1 above +h, 2 below -h
  T num = 0, den = 0;
  for (int i = 0; i < 3; i++, q /= 3) {
    const int st = q % 3;
    if (st == 0) continue;
    const T sg = st == 1 ? (T)1 : (T)-1;
    num += a[i] * (sg * h[i] - c[i]);
    den += a[i] * a[i];
  }
  if (!(den > minval<T>())) return false;
  s = num / den;
  return true;
}

template <typename T>
__device__ __forceinline__ T capsule_box_segpos(const T* c, const T* a, const T* h) {
  T e[3], p[3], s;
  const T hm = h[0] > h[1] ? (h[0] > h[2] ? h[0] : h[2]) : (h[1] > h[2] ? h[1] : h[2]);
  const T tol = (sizeof(T) == 8 ? (T)1e-10 : (T)1e-5) * ((T)1 + hm);
  // pass 1 also keeps a lower bound `other` on d over candidates at an s other than the argmin's:
  // when nothing else is within tol, the argmin is the answer and pass 2 is skipped
  T best = (T)1e30, sb = (T)2, other = (T)1e30;
  for (int k = 0; k < 49; k++) {
    if (!capsule_box_cand(k, c, a, h, s)) continue;
    s = clampv(s, (T)-1, (T)1);
    for (int i = 0; i < 3; i++) p[i] = c[i] + s * a[i];
    const T d = box_sd(p, h, e);
    if (d < best) {
      if (s != sb) other = best < other ? best : other;
      best = d;
      sb = s;
    } else if (s != sb) {
      other = d < other ? d : other;
    }
  }
  if (other > best + tol) return sb;
  T bs = (T)2;
  for (int k = 0; k < 49; k++) {
    if (!capsule_box_cand(k, c, a, h, s)) continue;
    s = clampv(s, (T)-1, (T)1);
    for (int i = 0; i < 3; i++) p[i] = c[i] + s * a[i];
    const T d = box_sd(p, h, e);
    if (d <= best + tol && s < bs) bs = s;
  }
  return bs;
}

// sphere of radius r at box-frame point pl (world point w) vs the box; e = outward face /
// feature normal in the box frame
template <typename T>
__device__ __forceinline__ int sphere_box_local(const T* pl, const T* w, T r, const T* bm, const T* h, T margin, T* e,
                                                Con<T>* out) {
  const T sd = box_sd(pl, h, e);
  const T dist = sd - r;
  if (dist > margin) return 0;
  T ew[3];
  mulmatvec3(ew, bm, e);
  out->dist = dist;
  for (int k = 0; k < 3; k++) { out->n[k] = -ew[k]; out->pos[k] = w[k] - ew[k] * (r + (T)0.5 * dist); }
  return 1;
}

// capsule (geom1) vs box (geom2), at most 2 contacts, structured as mjc_CapsuleBox [ext]: the axis
// point closest to / deepest in the box as a sphere-box contact; when that contact is on a box
// face, a second sphere-box contact at the far end of the axis's overlap with the face rectangle
// if that point is also within margin of the same face (a capsule lying along the face). The
// second point is dropped when it is within a tenth of the radius of the first.
template <typename T>
__device__ __forceinline__ int capsule_box(const T* cp, const T* cm, const T* cs, const T* bp, const T* bm, const T* h, T margin,
                           Con<T>* out) {
  const T r = cs[0], hl = cs[1];
  T tmp[3] = {cp[0] - bp[0], cp[1] - bp[1], cp[2] - bp[2]}, c[3], a[3];
  const T ax[3] = {cm[2] * hl, cm[5] * hl, cm[8] * hl};
  mulmatTvec3(c, bm, tmp);
  mulmatTvec3(a, bm, ax);
  const T s1 = capsule_box_segpos(c, a, h);
  T pl[3], w[3], e[3];
  for (int k = 0; k < 3; k++) { pl[k] = c[k] + s1 * a[k]; w[k] = cp[k] + s1 * ax[k]; }
  if (!sphere_box_local(pl, w, r, bm, h, margin, e, out)) return 0;
  int fk = -1, nz = 0;
  for (int k = 0; k < 3; k++)
    if (e[k] != 0) { nz++; fk = k; }
  if (nz != 1) return 1;  // edge or corner contact
  T lo = -1, hi = 1;
  for (int i = 0; i < 3; i++) {
    if (i == fk) continue;
    if (fabs(a[i]) > minval<T>()) {
      T t0 = (-h[i] - c[i]) / a[i], t1 = (h[i] - c[i]) / a[i];
      if (t0 > t1) { T t = t0; t0 = t1; t1 = t; }
      lo = t0 > lo ? t0 : lo;
      hi = t1 < hi ? t1 : hi;
    } else if (fabs(c[i]) > h[i]) {
      return 1;
    }
  }
  if (lo > hi) return 1;
  const T s2 = (s1 - lo < hi - s1) ? hi : lo;
  if (fabs(s2 - s1) * hl < (T)0.1 * r) return 1;
  T e2[3];
  for (int k = 0; k < 3; k++) { pl[k] = c[k] + s2 * a[k]; w[k] = cp[k] + s2 * ax[k]; }
  if (!sphere_box_local(pl, w, r, bm, h, margin, e2, out + 1)) return 1;
  // the far point must lie on the same face: one nonzero normal component, same axis and sign
  if ((e2[0] != 0) + (e2[1] != 0) + (e2[2] != 0) != 1 || !(e2[fk] * e[fk] > 0)) return 1;
  return 2;
}

// mjraw_SphereSphere [ext]: normal from 1 to 2; coincident centres take the cross product of the
// two geoms' z axes (then [1, 0, 0] when they are parallel)
template <typename T>
__device__ __forceinline__ int sph_sph_raw(const T* c1, const T* m1, T r1, const T* c2, const T* m2, T r2, T margin,
                                           Con<T>* out) {
  T dv[3] = {c2[0] - c1[0], c2[1] - c1[1], c2[2] - c1[2]};
  const T dist = sqrt(dot3(dv, dv)) - r1 - r2;
  if (dist > margin) return 0;
  const T L = normalize3(dv);
  if (L < minval<T>()) {
    const T z1[3] = {m1[2], m1[5], m1[8]}, z2[3] = {m2[2], m2[5], m2[8]};
    cross3(dv, z1, z2);
    normalize3(dv);
  }
  out->dist = dist;
  for (int k = 0; k < 3; k++) { out->n[k] = dv[k]; out->pos[k] = c1[k] + dv[k] * (r1 + (T)0.5 * dist); }
  return 1;
}

// mjc_CapsuleCapsule [ext]: closest points of the two axes in MuJoCo's centre + half-axis form
// (x1, x2 in [-1, 1], the same clamping sequence); for parallel axes (|det| < mjMINVAL) up to two
// sphere-sphere contacts from the axis ends (x1 = +-1, then x2 = +-1), stopping at two
template <typename T>
__device__ __forceinline__ int capsule_capsule(const T* p1, const T* m1, const T* s1, const T* p2, const T* m2, const T* s2,
                                               T margin, Con<T>* out) {
  const T a1[3] = {m1[2] * s1[1], m1[5] * s1[1], m1[8] * s1[1]};
  const T a2[3] = {m2[2] * s2[1], m2[5] * s2[1], m2[8] * s2[1]};
  const T dif[3] = {p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2]};
  const T ma = dot3(a1, a1), mb = -dot3(a1, a2), mc = dot3(a2, a2);
  const T u = -dot3(a1, dif), v = dot3(a2, dif);
  const T det = ma * mc - mb * mb;
  T v1[3], v2[3];
  if (fabs(det) >= minval<T>()) {
    T x1 = (mc * u - mb * v) / det, x2 = (ma * v - mb * u) / det;
    if (x1 > 1) { x1 = 1; x2 = (v - mb) / mc; }
    else if (x1 < -1) { x1 = -1; x2 = (v + mb) / mc; }
    if (x2 > 1) { x2 = 1; x1 = clampv((u - mb) / ma, (T)-1, (T)1); }
    else if (x2 < -1) { x2 = -1; x1 = clampv((u + mb) / ma, (T)-1, (T)1); }
    for (int k = 0; k < 3; k++) { v1[k] = p1[k] + a1[k] * x1; v2[k] = p2[k] + a2[k] * x2; }
    return sph_sph_raw(v1, m1, s1[0], v2, m2, s2[0], margin, out);
  }
  int n = 0;
  for (int e = 0; e < 4 && n < 2; e++) {
    const T sg = (e & 1) ? (T)-1 : (T)1;
    if (e < 2) {  // x1 = +-1
      const T x2 = clampv((v - sg * mb) / mc, (T)-1, (T)1);
      for (int k = 0; k < 3; k++) { v1[k] = p1[k] + sg * a1[k]; v2[k] = p2[k] + a2[k] * x2; }
    } else {      // x2 = +-1
      const T x1 = clampv((u - sg * mb) / ma, (T)-1, (T)1);
      for (int k = 0; k < 3; k++) { v1[k] = p1[k] + a1[k] * x1; v2[k] = p2[k] + sg * a2[k]; }
    }
    n += sph_sph_raw(v1, m1, s1[0], v2, m2, s2[0], margin, out + n);
  }
  return n;
}

// mjc_SphereCapsule [ext]: the sphere centre projected on the capsule axis, clamped to the
// half-length
template <typename T>
__device__ __forceinline__ int sphere_capsule(const T* p1, const T* m1, const T* s1, const T* p2, const T* m2, const T* s2,
                                              T margin, Con<T>* out) {
  const T ax[3] = {m2[2], m2[5], m2[8]};
  const T dv[3] = {p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2]};
  const T x = clampv(dot3(ax, dv), -s2[1], s2[1]);
  const T q[3] = {p2[0] + ax[0] * x, p2[1] + ax[1] * x, p2[2] + ax[2] * x};
  return sph_sph_raw(p1, m1, s1[0], q, m2, s2[0], margin, out);
}

// ---- cylinders (bipedal_rescue: sphere / capsule / box vs static cylinders) [ext]. MuJoCo
// sends these pairs through its general convex collider (one contact per pair); these are
// the oracle's closed forms on the exact (convex) cylinder signed distance (oracle/mjref.c).
template <typename T>
__device__ __forceinline__ T cyl_sd(const T* p, T r, T hh, T* e) {
  T rho = sqrt(p[0] * p[0] + p[1] * p[1]);
  T dr = rho - r, dz = fabs(p[2]) - hh;
  T ux = 1, uy = 0, sz = p[2] >= 0 ? (T)1 : (T)-1;
  if (rho > minval<T>()) { ux = p[0] / rho; uy = p[1] / rho; }
  if (dr > 0 && dz > 0) {
    T L = sqrt(dr * dr + dz * dz);
    e[0] = ux * dr / L; e[1] = uy * dr / L; e[2] = sz * dz / L;
    return L;
  }
  if (dr >= dz) { e[0] = ux; e[1] = uy; e[2] = 0; return dr; }
  e[0] = 0; e[1] = 0; e[2] = sz;
  return dz;
}

template <typename T>
__device__ __forceinline__ int sphere_cyl_core(const T* c, T R, const T* yp, const T* ym, const T* ys, T margin, Con<T>* out) {
  T tmp[3] = {c[0] - yp[0], c[1] - yp[1], c[2] - yp[2]}, pl[3], e[3], ew[3];
  mulmatTvec3(pl, ym, tmp);
  T dist = cyl_sd(pl, ys[0], ys[1], e) - R;
  if (dist > margin) return 0;
  mulmatvec3(ew, ym, e);
  out->dist = dist;
  for (int k = 0; k < 3; k++) { out->n[k] = -ew[k]; out->pos[k] = c[k] - ew[k] * (R + (T)0.5 * dist); }
  return 1;
}

template <typename T>
__device__ __forceinline__ int capsule_cyl(const T* cp, const T* cm, const T* cs, const T* yp, const T* ym, const T* ys, T margin,
                                           Con<T>* out) {
  T a[3], b[3], al[3], bl[3], tmp[3], e[3], p[3];
  seg_ends(cp, cm, cs[1], a, b);
  for (int k = 0; k < 3; k++) tmp[k] = a[k] - yp[k];
  mulmatTvec3(al, ym, tmp);
  for (int k = 0; k < 3; k++) tmp[k] = b[k] - yp[k];
  mulmatTvec3(bl, ym, tmp);
  T lo = 0, hi = 1;
  const T gr = (T)0.6180339887498949;
  T x1 = hi - gr * (hi - lo), x2 = lo + gr * (hi - lo), f1, f2;
  for (int k = 0; k < 3; k++) p[k] = al[k] + x1 * (bl[k] - al[k]);
  f1 = cyl_sd(p, ys[0], ys[1], e);
  for (int k = 0; k < 3; k++) p[k] = al[k] + x2 * (bl[k] - al[k]);
  f2 = cyl_sd(p, ys[0], ys[1], e);
  for (int it = 0; it < 40; it++) {
    if (f1 <= f2) {
      hi = x2; x2 = x1; f2 = f1; x1 = hi - gr * (hi - lo);
      for (int k = 0; k < 3; k++) p[k] = al[k] + x1 * (bl[k] - al[k]);
      f1 = cyl_sd(p, ys[0], ys[1], e);
    } else {
      lo = x1; x1 = x2; f1 = f2; x2 = lo + gr * (hi - lo);
      for (int k = 0; k < 3; k++) p[k] = al[k] + x2 * (bl[k] - al[k]);
      f2 = cyl_sd(p, ys[0], ys[1], e);
    }
  }
  T ts = (T)0.5 * (lo + hi);
  for (int k = 0; k < 3; k++) p[k] = al[k] + ts * (bl[k] - al[k]);
  T fs = cyl_sd(p, ys[0], ys[1], e), f0 = cyl_sd(al, ys[0], ys[1], e), fb = cyl_sd(bl, ys[0], ys[1], e);
  T t = ts;
  if (f0 <= fs && f0 <= fb) t = 0;
  else if (fb < fs) t = 1;
  T cw[3];
  for (int k = 0; k < 3; k++) cw[k] = a[k] + t * (b[k] - a[k]);
  return sphere_cyl_core(cw, cs[0], yp, ym, ys, margin, out);
}

template <typename T>
__device__ __forceinline__ int cyl_box(const T* yp, const T* ym, const T* ys, const T* bp, const T* bm, const T* h, T margin,
                                       Con<T>* out) {
  T best = (T)1e30, bn[3] = {0, 0, 1}, bpos[3] = {0, 0, 0};
  T v[3], w[3], tmp[3], pl[3], e[3], ew[3];
  for (int i = 0; i < 8; i++) {
    v[0] = (i & 1) ? h[0] : -h[0]; v[1] = (i & 2) ? h[1] : -h[1]; v[2] = (i & 4) ? h[2] : -h[2];
    mulmatvec3(w, bm, v);
    for (int k = 0; k < 3; k++) { w[k] += bp[k]; tmp[k] = w[k] - yp[k]; }
    mulmatTvec3(pl, ym, tmp);
    T sd = cyl_sd(pl, ys[0], ys[1], e);
    if (sd < best) {
      best = sd;
      mulmatvec3(ew, ym, e);
      for (int k = 0; k < 3; k++) { bn[k] = ew[k]; bpos[k] = w[k] - (T)0.5 * sd * ew[k]; }
    }
  }
  T q[3] = {yp[0], yp[1], yp[2]};
  for (int it = 0; it < 3; it++) {
    for (int k = 0; k < 3; k++) tmp[k] = q[k] - bp[k];
    mulmatTvec3(pl, bm, tmp);
    box_sd(pl, h, e);
    T d[3], dl[3];
    mulmatvec3(ew, bm, e);
    for (int k = 0; k < 3; k++) d[k] = -ew[k];
    mulmatTvec3(dl, ym, d);
    T rxy = sqrt(dl[0] * dl[0] + dl[1] * dl[1]);
    T sl[3] = {0, 0, dl[2] >= 0 ? ys[1] : -ys[1]};
    if (rxy > minval<T>()) { sl[0] = ys[0] * dl[0] / rxy; sl[1] = ys[0] * dl[1] / rxy; }
    mulmatvec3(q, ym, sl);
    for (int k = 0; k < 3; k++) q[k] += yp[k];
    for (int k = 0; k < 3; k++) tmp[k] = q[k] - bp[k];
    mulmatTvec3(pl, bm, tmp);
    T sd = box_sd(pl, h, e);
    if (sd < best) {
      best = sd;
      mulmatvec3(ew, bm, e);
      for (int k = 0; k < 3; k++) { bn[k] = -ew[k]; bpos[k] = q[k] - (T)0.5 * sd * ew[k]; }
    }
  }
  if (best > margin) return 0;
  out->dist = best;
  for (int k = 0; k < 3; k++) { out->n[k] = bn[k]; out->pos[k] = bpos[k]; }
  return 1;
}

template <typename T>
__device__ __forceinline__ int clip_poly(T (*in)[2], int n, int axis, T lim, T sgn, T tol, T (*out)[2]) {
  int m = 0;
  for (int i = 0; i < n; i++) {
    T* P = in[i];
    T* Q = in[(i + 1) % n];
    T dp = sgn * P[axis] - lim, dq = sgn * Q[axis] - lim;
    // a convex polygon gains at most one vertex per clip (4 -> 8 over the four clips); the
    // bound is also enforced, so a rounding-level non-convexity cannot write past out[8]
    if (dp <= tol && m < 8) { out[m][0] = P[0]; out[m][1] = P[1]; m++; }
    if (m < 8 && ((dp < -tol && dq > tol) || (dp > tol && dq < -tol))) {
      T t = dp / (dp - dq);
      out[m][0] = P[0] + t * (Q[0] - P[0]);
      out[m][1] = P[1] + t * (Q[1] - P[1]);
      m++;
    }
  }
  return m;
}

// Broadphase prefilters for scenes with many candidate pairs (collision(), DevModel.npair >
// MGX_TIGHT_BROADPHASE_PAIRS). Both are conservative: a pair they reject has no contact within its
// margin, so the narrowphase would return none and the contact list is unchanged; each test carries
// a slack of `tol` (relative to the geoms' sizes) so rounding can only let more pairs through.
// Two boxes separated along one of their six face axes by more than the margin: the face-axis
// part of box_box's separating-axis test.
template <typename T>
__device__ __forceinline__ bool box_box_separated(const T* pa, const T* Ra, const T* ha, const T* pb, const T* Rb,
                                                  const T* hb, T margin, T tol) {
  const T d[3] = {pb[0] - pa[0], pb[1] - pa[1], pb[2] - pa[2]};
  for (int ax = 0; ax < 6; ax++) {
    const T* R = ax < 3 ? Ra : Rb;
    const int c = ax < 3 ? ax : ax - 3;
    const T n[3] = {R[c], R[3 + c], R[6 + c]};  // the box's axis c (column c of its frame)
    T ra = 0, rb = 0;
    for (int k = 0; k < 3; k++) {
      ra += ha[k] * fabs(Ra[k] * n[0] + Ra[3 + k] * n[1] + Ra[6 + k] * n[2]);
      rb += hb[k] * fabs(Rb[k] * n[0] + Rb[3 + k] * n[1] + Rb[6 + k] * n[2]);
    }
    if (fabs(dot3(d, n)) - ra - rb > margin + tol * (ra + rb + (T)1)) return true;
  }
  return false;
}
// A geom within its bounding sphere (center c, radius r) against a box: the sphere is farther
// from the box than the margin.
template <typename T>
__device__ __forceinline__ bool sphere_box_separated(const T* c, T r, const T* pb, const T* Rb, const T* hb, T margin,
                                                     T tol) {
  const T v[3] = {c[0] - pb[0], c[1] - pb[1], c[2] - pb[2]};
  T d2 = 0;
  for (int k = 0; k < 3; k++) {
    const T q = Rb[k] * v[0] + Rb[3 + k] * v[1] + Rb[6 + k] * v[2];  // box frame
    const T o = fabs(q) - hb[k];
    if (o > 0) d2 += o * o;
  }
  const T lim = (r + margin) * ((T)1 + tol) + tol * (hb[0] + hb[1] + hb[2] + (T)1);
  return d2 > lim * lim;
}

template <typename T>
__device__ __forceinline__ int box_box(const T* pa, const T* Ra, const T* ha, const T* pb, const T* Rb, const T* hb, T margin,
                       Con<T>* out) {
  T d[3] = {pb[0] - pa[0], pb[1] - pa[1], pb[2] - pa[2]};
  T A[3][3], B[3][3];
  for (int i = 0; i < 3; i++)
    for (int k = 0; k < 3; k++) { A[i][k] = Ra[3 * k + i]; B[i][k] = Rb[3 * k + i]; }
  T best_face = (T)-1e30, best_edge = (T)-1e30;
  int face_axis = -1, edge_i = -1, edge_j = -1;
  // face-axis ties within ftol keep the earlier axis (oracle/mjref.c box_box)
  T hmax = 0;
  for (int k = 0; k < 3; k++) { hmax = ha[k] > hmax ? ha[k] : hmax; hmax = hb[k] > hmax ? hb[k] : hmax; }
  const T ftol = (T)1e-6 * hmax;
  T edge_n[3] = {0, 0, 0};
  for (int ax = 0; ax < 6; ax++) {
    const T* n = ax < 3 ? A[ax] : B[ax - 3];
    T ra = 0, rb = 0;
    for (int k = 0; k < 3; k++) { ra += ha[k] * fabs(dot3(A[k], n)); rb += hb[k] * fabs(dot3(B[k], n)); }
    T s = fabs(dot3(d, n)) - ra - rb;
    if (s > margin) return 0;
    if (s > best_face + ftol) { best_face = s; face_axis = ax; }
  }
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      T n[3];
      cross3(n, A[i], B[j]);
      T L = sqrt(dot3(n, n));
      if (L < (T)1e-6) continue;
      for (int k = 0; k < 3; k++) n[k] /= L;
      T ra = 0, rb = 0;
      for (int k = 0; k < 3; k++) { ra += ha[k] * fabs(dot3(A[k], n)); rb += hb[k] * fabs(dot3(B[k], n)); }
      T s = fabs(dot3(d, n)) - ra - rb;
      if (s > margin) return 0;
      if (s > best_edge) { best_edge = s; edge_i = i; edge_j = j; edge_n[0] = n[0]; edge_n[1] = n[1]; edge_n[2] = n[2]; }
    }
  if (edge_i >= 0 && best_edge > best_face + (T)1e-5 + (T)0.05 * fabs(best_face)) {
    T n[3] = {edge_n[0], edge_n[1], edge_n[2]};
    if (dot3(n, d) < 0) for (int k = 0; k < 3; k++) n[k] = -n[k];
    T ca[3] = {pa[0], pa[1], pa[2]}, cb[3] = {pb[0], pb[1], pb[2]};
    for (int k = 0; k < 3; k++) {
      if (k != edge_i) { T sg = dot3(A[k], n) >= 0 ? (T)1 : (T)-1; for (int c = 0; c < 3; c++) ca[c] += sg * ha[k] * A[k][c]; }
      if (k != edge_j) { T sg = dot3(B[k], n) <= 0 ? (T)1 : (T)-1; for (int c = 0; c < 3; c++) cb[c] += sg * hb[k] * B[k][c]; }
    }
    T a0[3], a1[3], b0[3], b1[3], s, t, P[3], Q[3];
    for (int c = 0; c < 3; c++) {
      a0[c] = ca[c] - ha[edge_i] * A[edge_i][c]; a1[c] = ca[c] + ha[edge_i] * A[edge_i][c];
      b0[c] = cb[c] - hb[edge_j] * B[edge_j][c]; b1[c] = cb[c] + hb[edge_j] * B[edge_j][c];
    }
    seg_seg(a0, a1, b0, b1, &s, &t);
    for (int c = 0; c < 3; c++) { P[c] = a0[c] + s * (a1[c] - a0[c]); Q[c] = b0[c] + t * (b1[c] - b0[c]); }
    T dq[3] = {Q[0] - P[0], Q[1] - P[1], Q[2] - P[2]};
    out[0].dist = dot3(dq, n);
    if (out[0].dist > margin) return 0;
    for (int c = 0; c < 3; c++) { out[0].n[c] = n[c]; out[0].pos[c] = (T)0.5 * (P[c] + Q[c]); }
    return 1;
  }
  // a NaN pose fails every separation test and leaves no axis selected: no contact (indexing with
  // face_axis = -1 read ha[-1] / hb[-1], one real before the model's geom_size slice, and A[-1];
  // round-6 fault audit). Finite poses always select an axis: results unchanged.
  if (face_axis < 0) return 0;
  bool refA = face_axis < 3;
  int ri = refA ? face_axis : face_axis - 3;
  const T* pr = refA ? pa : pb;
  const T* pi = refA ? pb : pa;
  const T* hr = refA ? ha : hb;
  const T* hi = refA ? hb : ha;
  T (*R)[3] = refA ? A : B;
  T (*I)[3] = refA ? B : A;
  T toI[3] = {pi[0] - pr[0], pi[1] - pr[1], pi[2] - pr[2]};
  T nr[3];
  T sg = dot3(toI, R[ri]) >= 0 ? (T)1 : (T)-1;
  for (int k = 0; k < 3; k++) nr[k] = sg * R[ri][k];
  int ii = 0;
  T bestd = -1;
  for (int k = 0; k < 3; k++) { T v = fabs(dot3(I[k], nr)); if (v > bestd) { bestd = v; ii = k; } }
  T si = dot3(I[ii], nr) > 0 ? (T)-1 : (T)1;
  T fc[3];
  for (int k = 0; k < 3; k++) fc[k] = pi[k] + si * hi[ii] * I[ii][k];
  int u = (ii + 1) % 3, v = (ii + 2) % 3;
  int ru = (ri + 1) % 3, rv = (ri + 2) % 3;
  T poly[8][2], tmp[8][2];
  const T sgn4[4][2] = {{1, 1}, {-1, 1}, {-1, -1}, {1, -1}};
  for (int c = 0; c < 4; c++) {
    T P[3], rel[3];
    for (int k = 0; k < 3; k++) P[k] = fc[k] + sgn4[c][0] * hi[u] * I[u][k] + sgn4[c][1] * hi[v] * I[v][k];
    for (int k = 0; k < 3; k++) rel[k] = P[k] - pr[k];
    poly[c][0] = dot3(rel, R[ru]);
    poly[c][1] = dot3(rel, R[rv]);
  }
  // vertices within tol of a clip line count as on it (oracle/mjref.c box_box)
  const T tol = (T)1e-5 * (hr[ru] > hr[rv] ? hr[ru] : hr[rv]);
  int np = 4;
  np = clip_poly(poly, np, 0, hr[ru], (T)1, tol, tmp);
  np = clip_poly(tmp, np, 0, hr[ru], (T)-1, tol, poly);
  np = clip_poly(poly, np, 1, hr[rv], (T)1, tol, tmp);
  np = clip_poly(tmp, np, 1, hr[rv], (T)-1, tol, poly);
  T fn[3];
  for (int k = 0; k < 3; k++) fn[k] = si * I[ii][k];
  T fndn = dot3(fn, nr);
  int n = 0;
  for (int c = 0; c < np && n < MGX_MAX_CONPAIR; c++) {
    T P[3];
    for (int k = 0; k < 3; k++) P[k] = pr[k] + poly[c][0] * R[ru][k] + poly[c][1] * R[rv][k] + hr[ri] * nr[k];
    T rel[3] = {P[0] - fc[0], P[1] - fc[1], P[2] - fc[2]};
    T t = fabs(fndn) > minval<T>() ? -dot3(rel, fn) / fndn : (T)0;
    if (t > margin) continue;
    out[n].dist = t;
    for (int k = 0; k < 3; k++) {
      out[n].n[k] = refA ? nr[k] : -nr[k];
      out[n].pos[k] = P[k] + (T)0.5 * t * nr[k];
    }
    n++;
  }
  return n;
}

template <typename T>
__device__ __forceinline__ int plane_sphere(const T* pp, const T* pm, const T* c, T r, T margin, Con<T>* out) {
  T n[3] = {pm[2], pm[5], pm[8]};
  T rel[3] = {c[0] - pp[0], c[1] - pp[1], c[2] - pp[2]};
  T dist = dot3(rel, n) - r;
  if (dist > margin) return 0;
  out->dist = dist;
  for (int k = 0; k < 3; k++) { out->n[k] = n[k]; out->pos[k] = c[k] - n[k] * (r + (T)0.5 * dist); }
  return 1;
}

template <typename T>
__device__ __forceinline__ int plane_box(const T* pp, const T* pm, const T* bp, const T* bm, const T* h, T margin, Con<T>* out) {
  T n[3] = {pm[2], pm[5], pm[8]};
  int cnt = 0;
  for (int c = 0; c < 8 && cnt < 4; c++) {
    T v[3], loc[3] = {(c & 1) ? h[0] : -h[0], (c & 2) ? h[1] : -h[1], (c & 4) ? h[2] : -h[2]};
    mulmatvec3(v, bm, loc);
    for (int k = 0; k < 3; k++) v[k] += bp[k];
    T rel[3] = {v[0] - pp[0], v[1] - pp[1], v[2] - pp[2]};
    T dist = dot3(rel, n);
    if (dist > margin) continue;
    out[cnt].dist = dist;
    for (int k = 0; k < 3; k++) { out[cnt].n[k] = n[k]; out[cnt].pos[k] = v[k] - (T)0.5 * dist * n[k]; }
    cnt++;
  }
  return cnt;
}

// cylinder support point in world direction d (oracle/mjref.c cyl_support)
template <typename T>
__device__ __forceinline__ void cyl_support(const T* yp, const T* ym, const T* ys, const T* d, T* q) {
  T dl[3];
  mulmatTvec3(dl, ym, d);
  T rxy = sqrt(dl[0] * dl[0] + dl[1] * dl[1]);
  T sl[3] = {0, 0, dl[2] >= 0 ? ys[1] : -ys[1]};
  if (rxy > minval<T>()) { sl[0] = ys[0] * dl[0] / rxy; sl[1] = ys[0] * dl[1] / rxy; }
  mulmatvec3(q, ym, sl);
  for (int k = 0; k < 3; k++) q[k] += yp[k];
}

template <typename T>
__device__ __forceinline__ T cyl_sd_world(const T* yp, const T* ym, const T* ys, const T* w, T* ew) {
  T tmp[3] = {w[0] - yp[0], w[1] - yp[1], w[2] - yp[2]}, pl[3], e[3];
  mulmatTvec3(pl, ym, tmp);
  T sd = cyl_sd(pl, ys[0], ys[1], e);
  mulmatvec3(ew, ym, e);
  return sd;
}

// cylinder (geom1) vs cylinder (geom2): fixed-point support search both ways, one contact
// (oracle/mjref.c cyl_cyl)
template <typename T>
__device__ __forceinline__ int cyl_cyl(const T* ap, const T* am, const T* as, const T* bp, const T* bm, const T* bs,
                                       T margin, Con<T>* out) {
  T best = (T)1e30, bn[3] = {0, 0, 1}, bpos[3] = {0, 0, 0};
  for (int side = 0; side < 2; side++) {
    const T *fp = side ? bp : ap, *fm = side ? bm : am, *fs = side ? bs : as;
    const T *sp = side ? ap : bp, *sm = side ? am : bm, *ss = side ? as : bs;
    T q[3] = {sp[0], sp[1], sp[2]}, ew[3], d[3];
    for (int it = 0; it < 4; it++) {
      cyl_sd_world(fp, fm, fs, q, ew);
      for (int k = 0; k < 3; k++) d[k] = -ew[k];
      cyl_support(sp, sm, ss, d, q);
      T sd = cyl_sd_world(fp, fm, fs, q, ew);
      if (sd < best) {
        best = sd;
        for (int k = 0; k < 3; k++) {
          bn[k] = side ? -ew[k] : ew[k];
          bpos[k] = q[k] - (T)0.5 * sd * ew[k];
        }
      }
    }
  }
  if (best > margin) return 0;
  out->dist = best;
  for (int k = 0; k < 3; k++) { out->n[k] = bn[k]; out->pos[k] = bpos[k]; }
  return 1;
}

// Dispatch one candidate pair. Geom frames come from LDS.
template <typename T>
__device__ __forceinline__ int collide_pair(int t1, int t2, const T* p1, const T* m1, const T* s1, const T* p2, const T* m2,
                            const T* s2, T margin, Con<T>* out) {
  if (t1 == GSPHERE && t2 == GSPHERE) return sph_sph_raw(p1, m1, s1[0], p2, m2, s2[0], margin, out);
  if (t1 == GSPHERE && t2 == GCAPSULE) return sphere_capsule(p1, m1, s1, p2, m2, s2, margin, out);
  if (t1 == GCAPSULE && t2 == GCAPSULE) return capsule_capsule(p1, m1, s1, p2, m2, s2, margin, out);
  if (t1 == GSPHERE && t2 == GBOX) return sphere_box_core(p1, s1[0], p2, m2, s2, margin, out);
  if (t1 == GCAPSULE && t2 == GBOX) return capsule_box(p1, m1, s1, p2, m2, s2, margin, out);
  if (t1 == GBOX && t2 == GBOX) return box_box(p1, m1, s1, p2, m2, s2, margin, out);
  if (t1 == GPLANE && t2 == GSPHERE) return plane_sphere(p1, m1, p2, s2[0], margin, out);
  if (t1 == GPLANE && t2 == GCAPSULE) {
    T a[3], b[3];
    seg_ends(p2, m2, s2[1], a, b);
    int n = plane_sphere(p1, m1, a, s2[0], margin, out);
    n += plane_sphere(p1, m1, b, s2[0], margin, out + n);
    return n;
  }
  if (t1 == GPLANE && t2 == GBOX) return plane_box(p1, m1, p2, m2, s2, margin, out);
  if (t1 == GSPHERE && t2 == GCYLINDER) return sphere_cyl_core(p1, s1[0], p2, m2, s2, margin, out);
  if (t1 == GCAPSULE && t2 == GCYLINDER) return capsule_cyl(p1, m1, s1, p2, m2, s2, margin, out);
  if (t1 == GCYLINDER && t2 == GBOX) return cyl_box(p1, m1, s1, p2, m2, s2, margin, out);
  if (t1 == GCYLINDER && t2 == GCYLINDER) return cyl_cyl(p1, m1, s1, p2, m2, s2, margin, out);
  return 0;
}

// mju_makeFrame: normal -> (normal, tangent1, tangent2)
template <typename T>
__device__ __forceinline__ void make_frame(T* f) {
  normalize3(f);
  f[3] = f[4] = f[5] = 0;
  if (f[1] < (T)0.5 && f[1] > (T)-0.5) f[4] = 1; else f[5] = 1;
  T s = dot3(f, f + 3);
  for (int k = 0; k < 3; k++) f[3 + k] -= f[k] * s;
  normalize3(f + 3);
  cross3(f + 6, f, f + 3);
}

}  // namespace mgx
