// scene.cpp -- scene-construction half of the C ABI (rt_xform_*, rt_scene_*, rt_shape_*)
// and the host flattener that turns the RayTracer-shaped rt_scene into the HBM layout of
// rt_blob.h.  Compiled with -ffp-contract=off: every precomputed value is produced with the
// same f64 op sequence the reference evaluates per call, so the device reads bit-equal data.
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <functional>
#include <new>
#include <string>
#include <vector>

#include "scene.h"

namespace rt {

static thread_local std::string g_last_error;

void set_error_message(const std::string& msg) { g_last_error = msg; }

int fail(int status, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return status;
}

// ---------------------------------------------------------------- transformations
// transformation.rs:208-220 -- accumulate from 0.0 in k order.
static void mat_mul(const double* a, const double* b, double* out) {
  double r[16];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      double acc = 0.0;
      for (int k = 0; k < 4; ++k) acc += a[4 * i + k] * b[4 * k + j];
      r[4 * i + j] = acc;
    }
  memcpy(out, r, sizeof r);
}

static void set_identity(double* m) {
  memset(m, 0, 16 * sizeof(double));
  m[0] = m[5] = m[10] = m[15] = 1.0;
}

void xf_identity(rt_transformation* t) {                       // :104-113
  set_identity(t->matrix);
  set_identity(t->inverse);
}

void xf_translation(double x, double y, double z, rt_transformation* t) {   // :164-180
  xf_identity(t);
  t->matrix[3] = x; t->matrix[7] = y; t->matrix[11] = z;
  t->inverse[3] = -x; t->inverse[7] = -y; t->inverse[11] = -z;
}

void xf_scaling(double x, double y, double z, rt_transformation* t) {      // :182-198
  xf_identity(t);
  t->matrix[0] = x; t->matrix[5] = y; t->matrix[10] = z;
  t->inverse[0] = 1.0 / x; t->inverse[5] = 1.0 / y; t->inverse[10] = 1.0 / z;
}

// Elementary rotations (:116-147); `axis` 0/1/2.
static void rotation_about(int axis, double angle, double* m) {
  double c = cos(angle), s = sin(angle);
  set_identity(m);
  if (axis == 0) { m[5] = c; m[6] = -s; m[9] = s; m[10] = c; }
  else if (axis == 1) { m[0] = c; m[2] = -s; m[8] = s; m[10] = c; }
  else { m[0] = c; m[1] = -s; m[4] = s; m[5] = c; }
}

void xf_rotation(double x, double y, double z, rt_transformation* t) {     // :115-162
  double m1[16], m2[16], m3[16], i1[16], i2[16], i3[16], tmp[16];
  rotation_about(0, x, m1); rotation_about(0, -x, i1);
  rotation_about(1, y, m2); rotation_about(1, -y, i2);
  rotation_about(2, z, m3); rotation_about(2, -z, i3);
  mat_mul(m1, m2, tmp); mat_mul(tmp, m3, t->matrix);
  mat_mul(i1, i2, tmp); mat_mul(tmp, i3, t->inverse);   // Rx(-x)Ry(-y)Rz(-z): the reference's "inverse"
}

void xf_compose(const rt_transformation& self, const rt_transformation& other, rt_transformation* out) {
  rt_transformation r;                                     // :200-205
  mat_mul(other.matrix, self.matrix, r.matrix);
  mat_mul(self.inverse, other.inverse, r.inverse);
  *out = r;
}

// transform_vector (:53-59): ((m0*x + m1*y) + m2*z) + m3 per row.
void xf_apply(const double m[16], const double v[3], double out[3]) {
  double a = m[0] * v[0] + m[1] * v[1] + m[2] * v[2] + m[3];
  double b = m[4] * v[0] + m[5] * v[1] + m[6] * v[2] + m[7];
  double c = m[8] * v[0] + m[9] * v[1] + m[10] * v[2] + m[11];
  out[0] = a; out[1] = b; out[2] = c;
}

// ---------------------------------------------------------------- small f64 vector helpers
struct V { double x, y, z; };
static inline double dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }         // vector.rs:94-100
static inline V scale(V a, double s) { return {a.x * s, a.y * s, a.z * s}; }
static inline V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static inline double length(V a) { return sqrt(dot(a, a)); }
static inline V normalized(V a) { return scale(a, 1.0 / length(a)); }                   // vector.rs:45-47
static inline V cross(V a, V b) {                                                        // vector.rs:61-67
  return {a.y * b.z - a.z * b.y, a.x * b.z - a.z * b.x, a.x * b.y - a.y * b.x};
}
static inline V apply(const double m[16], V v) {
  double in[3] = {v.x, v.y, v.z}, o[3];
  xf_apply(m, in, o);
  return {o[0], o[1], o[2]};
}
// transform_direction_vector (:70-77): T(v) - T(0)
static inline V apply_dir(const double m[16], V v) { return sub(apply(m, v), apply(m, {0.0, 0.0, 0.0})); }

// ---------------------------------------------------------------- flattening
static void leaf_common(const rt_transformation& t, RtLeaf* L) {
  memset(L, 0, sizeof *L);
  L->plane_axis = -1;
  memcpy(L->inv, t.inverse, 12 * sizeof(double));
  memcpy(L->mat, t.matrix, 12 * sizeof(double));
  V io = apply(t.inverse, {0.0, 0.0, 0.0});
  V mo = apply(t.matrix, {0.0, 0.0, 0.0});
  L->inv_o[0] = io.x; L->inv_o[1] = io.y; L->inv_o[2] = io.z;
  L->mat_o[0] = mo.x; L->mat_o[1] = mo.y; L->mat_o[2] = mo.z;
  // diagonal-affine inverse (rt_blob.h): off-diagonals +-0, all entries finite
  const double* m = t.inverse;
  bool diag = true;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 4; ++j) {
      const double v = m[4 * i + j];
      if (!std::isfinite(v)) diag = false;
      if (j < 3 && j != i && v != 0.0) diag = false;
    }
  const bool ident = diag && m[0] == 1.0 && m[5] == 1.0 && m[10] == 1.0 && m[3] == 0.0 && m[7] == 0.0 &&
                     m[11] == 0.0 && io.x == 0.0 && io.y == 0.0 && io.z == 0.0;
  L->xdiag = ident ? RT_XF_IDENTITY : diag ? 1 : 0;
}

// MathPlane::new (math_shapes.rs:140-152): raw (a,b,c,d) + transformed unit normal.
static void plane_into(const rt_transformation& t, double a, double b, double c, double d,
                       double pl[4], double pn[3]) {
  pl[0] = a; pl[1] = b; pl[2] = c; pl[3] = d;
  V n = normalized({a, b, c});
  V tn = normalized(apply_dir(t.matrix, n));                  // transformed_normal (:158-160)
  pn[0] = tn.x; pn[1] = tn.y; pn[2] = tn.z;
}

static int make_leaf(const ShapeRec& s, RtLeaf* L) {
  leaf_common(s.t, L);
  const double EPS = RT_EPSILON;
  switch (s.kind) {
    case SHAPE_SPHERE: {                                        // math_shapes.rs:28-39
      L->kind = RT_N_SPHERE;
      for (int i = 0; i < 3; ++i) L->c[i] = s.center[i];
      L->radius = s.size;
      L->r2 = s.size * s.size;
      L->r_eps = s.size + EPS;
      break;
    }
    case SHAPE_PLANE: {                                         // math_shapes.rs:154-156
      L->kind = RT_N_PLANE;
      plane_into(s.t, s.normal[0], s.normal[1], s.normal[2], s.distance, L->pl[0], L->pn[0]);
      V pn = normalized({s.normal[0], s.normal[1], s.normal[2]});   // intersects (:169)
      L->pnorm[0] = pn.x; L->pnorm[1] = pn.y; L->pnorm[2] = pn.z;
      {
        const double n[3] = {pn.x, pn.y, pn.z};
        int nz = 0, ax = -1;
        for (int i = 0; i < 3; ++i)
          if (n[i] != 0.0) { ++nz; ax = i; }
        // untransformed planes only: the kernel's `fin` is the finiteness of the WORLD ray, which is
        // the object-space ray only under the identity (a transform may overflow to inf)
        L->plane_axis = (nz == 1 && std::isfinite(n[ax]) && L->xdiag == RT_XF_IDENTITY) ? ax : -1;
      }
      break;
    }
    case SHAPE_CUBE: {                                          // math_shapes.rs:228-244
      L->kind = RT_N_CUBE;
      double length = s.size / 2.0;
      const double* c = s.center;
      for (int i = 0; i < 3; ++i) {
        L->c[i] = c[i];
        L->lo[i] = c[i] - length;
        L->hi[i] = c[i] + length;
        L->lo_e[i] = c[i] - length - EPS;
        L->hi_e[i] = c[i] + length + EPS;
      }
      L->radius = length;
      // stored in get_normal order p1..p6 (:298-305); note the planes sit at +-length/2 (quirk)
      plane_into(s.t, 0.0, 0.0, 1.0, -(c[2] + length / 2.0), L->pl[0], L->pn[0]);   // p1
      plane_into(s.t, 0.0, 1.0, 0.0, -(c[1] + length / 2.0), L->pl[1], L->pn[1]);   // p2
      plane_into(s.t, 1.0, 0.0, 0.0, -(c[0] + length / 2.0), L->pl[2], L->pn[2]);   // p3
      plane_into(s.t, -1.0, 0.0, 0.0, c[0] + -length / 2.0, L->pl[3], L->pn[3]);    // p4
      plane_into(s.t, 0.0, -1.0, 0.0, c[1] + -length / 2.0, L->pl[4], L->pn[4]);    // p5
      plane_into(s.t, 0.0, 0.0, -1.0, c[2] + -length / 2.0, L->pl[5], L->pn[5]);    // p6
      break;
    }
    default:
      return fail(RT_ERR_INVALID, "internal: make_leaf on CSG");
  }
  return RT_OK;
}

// ---------------------------------------------------------------- culling bounds
// World-space AABB of the region {p : Minv * p in B} for an object-space ball / box B.  The
// reference tests points through the INVERSE matrix (which for multi-axis rotations is not the
// exact inverse of the forward matrix, transformation.rs:149-159), so the region is the image of
// B under Minv^-1, computed here in long double and inflated generously.
struct Box { double lo[3], hi[3]; int kind; };   // kind: RtCull

static Box box_infinite() { Box b; for (int i = 0; i < 3; ++i) { b.lo[i] = -INFINITY; b.hi[i] = INFINITY; } b.kind = RT_CULL_NONE; return b; }
static Box box_empty() { Box b; for (int i = 0; i < 3; ++i) { b.lo[i] = INFINITY; b.hi[i] = -INFINITY; } b.kind = RT_CULL_ALWAYS; return b; }

static Box box_hull(const Box& a, const Box& b) {
  if (a.kind == RT_CULL_ALWAYS) return b;
  if (b.kind == RT_CULL_ALWAYS) return a;
  if (a.kind == RT_CULL_NONE || b.kind == RT_CULL_NONE) return box_infinite();
  Box r;
  r.kind = RT_CULL_BOX;
  for (int i = 0; i < 3; ++i) { r.lo[i] = fmin(a.lo[i], b.lo[i]); r.hi[i] = fmax(a.hi[i], b.hi[i]); }
  return r;
}
static Box box_meet(const Box& a, const Box& b) {
  if (a.kind == RT_CULL_ALWAYS || b.kind == RT_CULL_ALWAYS) return box_empty();
  if (a.kind == RT_CULL_NONE) return b;
  if (b.kind == RT_CULL_NONE) return a;
  Box r;
  r.kind = RT_CULL_BOX;
  for (int i = 0; i < 3; ++i) {
    r.lo[i] = fmax(a.lo[i], b.lo[i]);
    r.hi[i] = fmin(a.hi[i], b.hi[i]);
    if (r.lo[i] > r.hi[i]) return box_empty();
  }
  return r;
}

// Leaf's own region (points its hits and its is_inside can involve), in world space.
static Box leaf_box(const ShapeRec& s) {
  if (s.kind == SHAPE_PLANE) return box_infinite();
  const double* iv = s.t.inverse;
  long double A[3][3], b[3], Ai[3][3];
  for (int i = 0; i < 3; ++i) { for (int j = 0; j < 3; ++j) A[i][j] = iv[4 * i + j]; b[i] = iv[4 * i + 3]; }
  long double det = A[0][0] * (A[1][1] * A[2][2] - A[1][2] * A[2][1]) - A[0][1] * (A[1][0] * A[2][2] - A[1][2] * A[2][0]) +
                    A[0][2] * (A[1][0] * A[2][1] - A[1][1] * A[2][0]);
  if (!(fabsl(det) > 1e-300L) || !isfinite((double)det)) return box_infinite();
  Ai[0][0] = (A[1][1] * A[2][2] - A[1][2] * A[2][1]) / det;
  Ai[0][1] = (A[0][2] * A[2][1] - A[0][1] * A[2][2]) / det;
  Ai[0][2] = (A[0][1] * A[1][2] - A[0][2] * A[1][1]) / det;
  Ai[1][0] = (A[1][2] * A[2][0] - A[1][0] * A[2][2]) / det;
  Ai[1][1] = (A[0][0] * A[2][2] - A[0][2] * A[2][0]) / det;
  Ai[1][2] = (A[0][2] * A[1][0] - A[0][0] * A[1][2]) / det;
  Ai[2][0] = (A[1][0] * A[2][1] - A[1][1] * A[2][0]) / det;
  Ai[2][1] = (A[0][1] * A[2][0] - A[0][0] * A[2][1]) / det;
  Ai[2][2] = (A[0][0] * A[1][1] - A[0][1] * A[1][0]) / det;
  const long double eps = RT_EPSILON;
  long double c[3], half[3];
  for (int i = 0; i < 3; ++i) c[i] = (long double)s.center[i] - b[i];
  Box r;
  r.kind = RT_CULL_BOX;
  for (int i = 0; i < 3; ++i) {
    long double wc = Ai[i][0] * c[0] + Ai[i][1] * c[1] + Ai[i][2] * c[2];
    if (s.kind == SHAPE_SPHERE) {                 // ball of radius r (+EPS: is_inside's slack)
      long double rad = fabsl((long double)s.size) + eps;
      half[i] = rad * sqrtl(Ai[i][0] * Ai[i][0] + Ai[i][1] * Ai[i][1] + Ai[i][2] * Ai[i][2]);
    } else {                                      // box of half-length size/2 (+EPS)
      long double h = fabsl((long double)s.size / 2.0L) + eps;
      half[i] = h * (fabsl(Ai[i][0]) + fabsl(Ai[i][1]) + fabsl(Ai[i][2]));
    }
    long double margin = 1e-6L * (fabsl(wc) + half[i]) + 1e-6L;
    r.lo[i] = (double)(wc - half[i] - margin);
    r.hi[i] = (double)(wc + half[i] + margin);
    // the kernel's slab arithmetic is only proven conservative for coordinates within 1e6
    // (rt_device.h cull_ray): larger boxes are never culled
    if (!(fabs(r.lo[i]) <= RT_CULL_COORD_MAX) || !(fabs(r.hi[i]) <= RT_CULL_COORD_MAX)) return box_infinite();
  }
  return r;
}

struct Flattener {
  const rt_scene& s;
  FlatScene& f;
  int32_t node_begin = 0;
  std::vector<int32_t> parent;         // per node (object-relative): parent node or -1
  std::vector<Box> box;                // per node (object-relative): region of its is_inside / hits
  int depth_guard = 0;

  // Emit the subtree of shape id `sid`; returns its object-relative node index.
  int32_t emit(int32_t sid, int* err) {
    if (sid < 0 || sid >= (int32_t)s.shapes.size()) { *err = fail(RT_ERR_INVALID, "bad shape id %d", sid); return -1; }
    if (++depth_guard > 64) { *err = fail(RT_ERR_UNSUPPORTED, "CSG nesting deeper than 64"); return -1; }
    const ShapeRec& r = s.shapes[sid];
    RtNode n;
    memset(&n, 0, sizeof n);
    if (r.kind == SHAPE_CSG) {
      int32_t a = emit(r.a, err);
      if (*err) return -1;
      int32_t b = emit(r.b, err);
      if (*err) return -1;
      n.kind = r.op == RT_CSG_UNION ? RT_N_UNION : r.op == RT_CSG_INTERSECTION ? RT_N_INTERSECTION : RT_N_DIFFERENCE;
      n.a = a; n.b = b; n.leaf = -1;
    } else {
      RtLeaf L;
      int rc = make_leaf(r, &L);
      if (rc) { *err = rc; return -1; }
      n.kind = L.kind; n.a = n.b = -1;
      n.leaf = (int32_t)f.leaves.size();
      f.leaves.push_back(L);
    }
    --depth_guard;
    int32_t idx = (int32_t)f.nodes.size() - node_begin;
    f.nodes.push_back(n);
    parent.push_back(-1);
    if (n.kind >= RT_N_UNION) {
      parent[n.a] = idx; parent[n.b] = idx;
      // csg.rs:126-135: union -> either child, intersection -> both, difference -> inside a
      box.push_back(n.kind == RT_N_UNION ? box_hull(box[n.a], box[n.b])
                    : n.kind == RT_N_INTERSECTION ? box_meet(box[n.a], box[n.b]) : box[n.a]);
    } else {
      box.push_back(leaf_box(r));
    }
    return idx;
  }

  // postfix is_inside of subtree rooted at object-relative node `ni` (csg.rs:126-135)
  void emit_inside(int32_t ni) {
    const RtNode& n = f.nodes[node_begin + ni];
    if (n.kind < RT_N_UNION) { f.prog.push_back({RT_OP_INSIDE, n.leaf}); return; }
    emit_inside(n.a);
    emit_inside(n.b);
    int32_t op = n.kind == RT_N_UNION ? RT_OP_OR : n.kind == RT_N_INTERSECTION ? RT_OP_AND : RT_OP_ANDNOT;
    f.prog.push_back({op, 0});
  }
};

// Two sphere leaves with bit-identical inverse transforms and centres: the same object-space ray
// for every world ray, hence the same 1/|d|, v.dn and v.v (rt_blob.h share_prev).
static bool shares_sphere_terms(const RtLeaf& L, const RtLeaf& P) {
  return L.kind == RT_N_SPHERE && P.kind == RT_N_SPHERE && L.xdiag == P.xdiag && !memcmp(L.inv, P.inv, sizeof L.inv) &&
         !memcmp(L.inv_o, P.inv_o, sizeof L.inv_o) && !memcmp(L.c, P.c, sizeof L.c);
}

// ---------------------------------------------------------------- hit-filter literal form
// Rewrite a leaf's postfix filter program [b, e) into a conjunction of literals (2*leaf + want)
// when every REQUIRE reduces to one: v == 1 of AND / ANDNOT and v == 0 of OR distribute over
// their operands; anything else (a disjunction) keeps the program.  Returns the literal count,
// or -1.
static int filter_literals(const std::vector<RtProg>& prog, int32_t b, int32_t e, int32_t* lits) {
  struct Fm { int32_t op, leaf, a, b; };
  std::vector<Fm> fm;
  std::vector<int32_t> st;
  std::vector<int32_t> out;
  bool ok = true;
  std::function<void(int32_t, int32_t)> conj = [&](int32_t x, int32_t want) {
    const Fm& f = fm[x];
    if (f.op == RT_OP_INSIDE) { out.push_back(2 * f.leaf + want); return; }
    if (want == 1 && f.op == RT_OP_AND) { conj(f.a, 1); conj(f.b, 1); return; }
    if (want == 1 && f.op == RT_OP_ANDNOT) { conj(f.a, 1); conj(f.b, 0); return; }
    if (want == 0 && f.op == RT_OP_OR) { conj(f.a, 0); conj(f.b, 0); return; }
    ok = false;
  };
  for (int32_t k = b; k < e && ok; ++k) {
    const RtProg& p = prog[k];
    if (p.op == RT_OP_INSIDE) {
      fm.push_back({RT_OP_INSIDE, p.arg, -1, -1});
      st.push_back((int32_t)fm.size() - 1);
    } else if (p.op == RT_OP_REQUIRE) {
      if (st.empty()) return -1;
      conj(st.back(), p.arg);
      st.pop_back();
    } else {
      if (st.size() < 2) return -1;
      const int32_t y = st.back(); st.pop_back();
      const int32_t x = st.back(); st.pop_back();
      fm.push_back({p.op, -1, x, y});
      st.push_back((int32_t)fm.size() - 1);
    }
  }
  if (!ok || !st.empty()) return -1;
  std::vector<int32_t> uniq;
  for (int32_t v : out)
    if (std::find(uniq.begin(), uniq.end(), v) == uniq.end()) uniq.push_back(v);
  if (uniq.size() > RT_MAX_LITS) return -1;
  for (size_t i = 0; i < uniq.size(); ++i) lits[i] = uniq[i];
  return (int32_t)uniq.size();
}

// Concentric sphere leaves with one transform share their ray terms (rt_blob.h share_prev).  The
// refraction kernels use the shared terms (rt_device.h trace: SHARE), so in scenes with a
// transparent object per-leaf box tests that cannot cull, or that cost what the shared quadratic
// costs, are dropped as well.  `uncond`: the leaf is evaluated whenever its object is entered.
static void share_sphere_terms(FlatScene& f, RtObject* ob) {
  if (ob->leaf_cull && f.any_transparent) {
    bool prev_uncond = false;
    for (int32_t l = ob->leaf_begin; l < ob->leaf_begin + ob->leaf_count; ++l) {
      RtLeaf& L = f.leaves[l];
      bool uncond = L.cull == RT_CULL_NONE;
      // the first leaf's test repeats the object's (same box, same tmax: no hit accepted between)
      if (l == ob->leaf_begin && L.cull == RT_CULL_BOX && ob->cull == RT_CULL_BOX &&
          !memcmp(L.blo, ob->blo, sizeof L.blo) && !memcmp(L.bhi, ob->bhi, sizeof L.bhi)) {
        L.cull = RT_CULL_NONE;
        uncond = true;
      }
      // a sharing sphere whose predecessor always runs: its test costs what the shared quadratic
      // costs (a ray that misses the sphere stops at `sum < 0`), so it runs unconditionally too
      if (l > ob->leaf_begin && prev_uncond && L.cull == RT_CULL_BOX && shares_sphere_terms(L, f.leaves[l - 1])) {
        L.cull = RT_CULL_NONE;
        uncond = true;
      }
      prev_uncond = uncond;
    }
    bool any_test = false;
    for (int32_t l = ob->leaf_begin; l < ob->leaf_begin + ob->leaf_count; ++l) any_test |= f.leaves[l].cull != RT_CULL_NONE;
    ob->leaf_cull = any_test;
  }
  for (int32_t l = ob->leaf_begin + 1; l < ob->leaf_begin + ob->leaf_count; ++l) {
    RtLeaf& L = f.leaves[l];
    const RtLeaf& P = f.leaves[l - 1];
    L.share_prev = 0;
    if (!shares_sphere_terms(L, P)) continue;
    bool inner = L.cull == RT_CULL_BOX && P.cull == RT_CULL_BOX;
    for (int i = 0; i < 3 && inner; ++i) inner = P.blo[i] <= L.blo[i] && L.bhi[i] <= P.bhi[i];
    if (!ob->leaf_cull || P.cull == RT_CULL_NONE || L.cull == RT_CULL_ALWAYS || inner) L.share_prev = 1;
  }
}

// ---------------------------------------------------------------- hit-filter literal order
// A literal filter is a conjunction of pure tests, so its order is free (the kernels stop at the
// first failing literal).  Most likely failures first: for a hit of leaf X, "inside R" fails about
// 1 - vol(R)/vol(X) of the time and "not inside R" about vol(R)/vol(X) (world volumes of the
// leaves' regions); for spheres sharing X's transform and centre the answer is known from the radii
// (globes.scene's claw: a hit on the outer shell is never inside the inner one, but is usually
// outside the thin slab, so the slab test goes first).
static double leaf_world_volume(const RtLeaf& L) {
  const double* M = L.inv;
  const double det = M[0] * (M[5] * M[10] - M[6] * M[9]) - M[1] * (M[4] * M[10] - M[6] * M[8]) +
                     M[2] * (M[4] * M[9] - M[5] * M[8]);
  const double v = L.kind == RT_N_SPHERE ? 4.18879020478639 * L.radius * L.radius * L.radius
                 : L.kind == RT_N_CUBE ? 8.0 * L.radius * L.radius * L.radius : INFINITY;
  return std::isfinite(det) && det != 0.0 ? fabs(v / det) : INFINITY;
}

static void order_literals(FlatScene& f, const RtObject& ob) {
  for (int32_t x = ob.leaf_begin; x < ob.leaf_begin + ob.leaf_count; ++x) {
    RtLeaf& X = f.leaves[x];
    if (X.n_lit < 2) continue;
    const double vx = leaf_world_volume(X);
    double fail[RT_MAX_LITS];
    for (int k = 0; k < X.n_lit; ++k) {
      const RtLeaf& R = f.leaves[X.lit[k] >> 1];
      const bool want = X.lit[k] & 1;
      if (X.kind == RT_N_SPHERE && R.kind == RT_N_SPHERE && shares_sphere_terms(X, R)) {
        fail[k] = want ? (X.radius < R.radius ? 0.0 : 1.0) : (X.radius > R.radius ? 0.0 : 1.0);
        continue;
      }
      const double vr = leaf_world_volume(R);
      const double frac = std::isfinite(vx) && std::isfinite(vr) && vx > 0.0 ? std::min(1.0, vr / vx) : 0.5;
      fail[k] = want ? 1.0 - frac : frac;
    }
    int idx[RT_MAX_LITS];
    for (int k = 0; k < X.n_lit; ++k) idx[k] = k;
    std::stable_sort(idx, idx + X.n_lit, [&](int a, int b) { return fail[a] > fail[b]; });
    int32_t lits[RT_MAX_LITS];
    for (int k = 0; k < X.n_lit; ++k) lits[k] = X.lit[idx[k]];
    if (!diag_env("RT_NO_LIT_ORDER"))
      for (int k = 0; k < X.n_lit; ++k) X.lit[k] = lits[k];
  }
}

// ---------------------------------------------------------------- constant hit filters
// A hit of sphere X tested against a sphere R with the same transform and centre (bit-identical
// inv, inv_o, c): the filter's point q = xf(inv, o + t d) lies at |q - c| = r_X up to rounding in
// the quadratic's t, the world point and the transform, all below ~1e-14 (1 + |M|) (|o| + |p| +
// |T| + |c| + r) -- |p| is bounded by the sphere's world extent, and the traversals only skip the
// filter for ray origins |o| <= 1e6 (their culling ray's range, rt_device.h cull_ray).  With
// the margin m below (>= 1e6 x that bound) "inside R" (|q - c| <= r_R + EPS) is always true when
// r_X + m < r_R and always false when r_X - m > r_R + EPS: spinning_globes.scene's glass shells,
// globes.scene's claw.  A filter whose every literal always passes is skipped (filter_const).
static void const_filters(FlatScene& f, const RtObject& ob) {
  for (int32_t x = ob.leaf_begin; x < ob.leaf_begin + ob.leaf_count; ++x) {
    RtLeaf& X = f.leaves[x];
    X.filter_const = 0;
    if (X.kind != RT_N_SPHERE || X.n_lit < 1 || diag_env("RT_NO_CONST_FILTER")) continue;
    double mrow = 0.0, fwd = 0.0, tsum = 0.0;
    for (int i = 0; i < 3; ++i) {
      mrow = std::max(mrow, fabs(X.inv[4 * i]) + fabs(X.inv[4 * i + 1]) + fabs(X.inv[4 * i + 2]));
      fwd = std::max(fwd, fabs(X.mat[4 * i]) + fabs(X.mat[4 * i + 1]) + fabs(X.mat[4 * i + 2]));
      tsum += fabs(X.inv[4 * i + 3]) + fabs(X.inv_o[i]) + fabs(X.mat[4 * i + 3]) + fabs(X.c[i]);
    }
    bool all = true;
    for (int k = 0; k < X.n_lit && all; ++k) {
      const RtLeaf& R = f.leaves[X.lit[k] >> 1];
      const bool want = X.lit[k] & 1;
      if (R.kind != RT_N_SPHERE || !shares_sphere_terms(X, R)) { all = false; break; }
      const double extent = fwd * (tsum + X.radius + R.radius) + tsum;     // bounds |p| for hits of X
      const double m = 1e-8 * (1.0 + mrow) * (1e6 + extent + tsum + X.radius + R.radius);
      const bool finite = std::isfinite(m) && std::isfinite(X.radius) && std::isfinite(R.r_eps);
      all = finite && (want ? X.radius + m < R.radius : X.radius - m > R.r_eps);
    }
    X.filter_const = all ? 1 : 0;
  }
}

// ---------------------------------------------------------------- oriented object boxes
// An object's accepted hits all lie inside leaf R's region when, for every leaf X of the object,
// X is R or X's hit filter requires inside(R) (a literal 2R+1): a hit of R itself lies on R's
// surface, any other accepted hit passed R's is_inside test.  R's region is a box in R's own
// frame (sphere: centre +- (r + EPS), cube: [lo, hi]), so a ray whose image under R's inverse
// transform misses that box cannot produce an accepted hit of the object.  The kernels test it
// after the world box (rt_device.h obb_may_hit) when its world volume is under half the
// world box's -- e.g. globes.scene's tilted axis rod and thin claw slab.
//
// Margins (local units, per axis i, on top of the box): the kernel forms o' = xf(inv, o) and
// d' = xf(inv, d) - inv_o exactly as the leaves do, so R's own hits are at the same o' + t d';
// other leaves' hits were tested at q = xf(inv, p), p = o + t d.  Their difference is rounding:
// <= ~4 ulp of (|M_i| |p| + |T_i|) for q, the same for o', and t times ~2 ulp of
// (|M_i| |d| + |T_i|) for d' (the - inv_o cancels T).  The kernel only takes the test for
// |o| <= 1e6 and |d|_max in [1/4, 4] (unit-length directions), and |p| <= 1e6 inside the world
// box, so t <= 8e6 and the error is < 1e-8 (|M_i| + |T_i|); the margin is 1e-6 (1 + |M_i| + |T_i|)
// plus 1e-6 of the box coordinates, and the slab arithmetic itself is the world box test's
// (cull_ray / box_may_hit).
static void obb(FlatScene& f, RtObject* ob) {
  ob->obb_leaf = -1;
  if (ob->cull != RT_CULL_BOX || diag_env("RT_NO_OBB")) return;
  double wvol = 1.0;
  for (int i = 0; i < 3; ++i) wvol *= ob->bhi[i] - ob->blo[i];
  double best = 0.5 * wvol;
  for (int32_t r = ob->leaf_begin; r < ob->leaf_begin + ob->leaf_count; ++r) {
    const RtLeaf& R = f.leaves[r];
    if (R.kind != RT_N_SPHERE && R.kind != RT_N_CUBE) continue;
    bool all = true;
    for (int32_t x = ob->leaf_begin; x < ob->leaf_begin + ob->leaf_count && all; ++x) {
      if (x == r) continue;
      const RtLeaf& X = f.leaves[x];
      bool req = false;
      for (int k = 0; k < X.n_lit && !req; ++k) req = X.lit[k] == 2 * r + 1;
      all = req;                       // n_lit < 0 (a disjunctive filter): never required
    }
    if (!all) continue;
    double lo[3], hi[3];
    for (int i = 0; i < 3; ++i) {
      lo[i] = R.kind == RT_N_SPHERE ? R.c[i] - R.r_eps : R.lo[i];
      hi[i] = R.kind == RT_N_SPHERE ? R.c[i] + R.r_eps : R.hi[i];
    }
    const double* M = R.inv;
    const double det = M[0] * (M[5] * M[10] - M[6] * M[9]) - M[1] * (M[4] * M[10] - M[6] * M[8]) +
                       M[2] * (M[4] * M[9] - M[5] * M[8]);
    if (!std::isfinite(det) || !(fabs(det) > 1e-300)) continue;
    bool ok = true;
    double vol = 1.0;
    for (int i = 0; i < 3 && ok; ++i) {
      const double mi = fabs(M[4 * i]) + fabs(M[4 * i + 1]) + fabs(M[4 * i + 2]), ti = fabs(M[4 * i + 3]) + fabs(R.inv_o[i]);
      const double m = 1e-6 * (1.0 + mi + ti) + 1e-6 * (fabs(lo[i]) + fabs(hi[i]));
      lo[i] -= m;
      hi[i] += m;
      ok = std::isfinite(lo[i]) && std::isfinite(hi[i]) && fabs(lo[i]) <= RT_CULL_COORD_MAX && fabs(hi[i]) <= RT_CULL_COORD_MAX;
      vol *= hi[i] - lo[i];
    }
    if (!ok) continue;
    vol /= fabs(det);                  // world volume of the local box
    if (vol < best) {
      best = vol;
      ob->obb_leaf = r;
      for (int i = 0; i < 3; ++i) { ob->olo[i] = lo[i]; ob->ohi[i] = hi[i]; }
    }
  }
}

// ---------------------------------------------------------------- constant normals
// A plane object's normal is its leaf's constant MathPlane::normal; get_ray_color normalises it
// (raytracer.rs:163) and every angle divides by its length (vector.rs:57-59).  The kernels' normalized()
// and len() are IEEE sqrt / division / products in this order (rt_device.h: sqrt_core and recip_core
// are bit-identical to sqrt and 1.0 / l), so the host forms both once.  Only finite results are kept.
static void unit_normal(const FlatScene& f, RtObject* ob) {
  ob->unit_normal = 0;
  if (ob->node_count != 1 || diag_env("RT_NO_UNIT_NORMAL")) return;
  const RtLeaf& L = f.leaves[ob->leaf_begin];
  if (L.kind != RT_N_PLANE) return;
  const double* a = L.pn[0];
  const double x = (a[0] * a[0] + a[1] * a[1]) + a[2] * a[2];
  const double l = sqrt(x), il = 1.0 / l;
  const double n[3] = {a[0] * il, a[1] * il, a[2] * il};
  const double nl = sqrt((n[0] * n[0] + n[1] * n[1]) + n[2] * n[2]);
  if (!(std::isfinite(n[0]) && std::isfinite(n[1]) && std::isfinite(n[2]) && std::isfinite(nl) && nl > 0.0)) return;
  for (int i = 0; i < 3; ++i) ob->nunit[i] = n[i];
  ob->nunit_len = nl;
  ob->unit_normal = 1;
}

// ---------------------------------------------------------------- object hierarchy
static double box_area(const double* lo, const double* hi) {
  const double x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
  return 2.0 * (x * y + y * z + z * x);
}

struct HierBuilder {
  FlatScene& f;
  std::vector<RtTrav>& out;
  const std::vector<int>& perm;        // position -> object index
  void hull(int a, int b, double* lo, double* hi) const {
    for (int k = 0; k < 3; ++k) { lo[k] = INFINITY; hi[k] = -INFINITY; }
    for (int o = a; o < b; ++o)
      for (int k = 0; k < 3; ++k) {
        lo[k] = fmin(lo[k], f.objects[perm[o]].blo[k]);
        hi[k] = fmax(hi[k], f.objects[perm[o]].bhi[k]);
      }
  }
  void object(int o) {
    RtTrav t;
    memset(&t, 0, sizeof t);
    t.obj = perm[o];
    t.skip = (int32_t)out.size() + 1;
    const RtObject& ob = f.objects[perm[o]];
    for (int k = 0; k < 3; ++k) { t.blo[k] = ob.blo[k]; t.bhi[k] = ob.bhi[k]; }
    t.cull = ob.cull;
    t.shadow_skip = ob.shadow_skip;
    out.push_back(t);
  }
  // Positions [a, b), all objects with a finite box.  A group node is emitted when it is clearly
  // smaller than the enclosing group (surface area); the run is split where the SAH cost is lowest.
  void run(int a, int b, double parent_area) {
    if (b - a == 1) { object(a); return; }
    RtTrav g;
    memset(&g, 0, sizeof g);
    hull(a, b, g.blo, g.bhi);
    const double area = box_area(g.blo, g.bhi);
    const bool group = area <= 0.8 * parent_area;
    const size_t gi = out.size();
    if (group) { g.obj = -1; out.push_back(g); parent_area = area; }
    if (b - a == 2) {
      object(a);
      object(a + 1);
    } else {
      int best_k = a + 1;
      double best = INFINITY;
      for (int k = a + 1; k < b; ++k) {
        double lo[3], hi[3], lo2[3], hi2[3];
        hull(a, k, lo, hi);
        hull(k, b, lo2, hi2);
        const double cost = box_area(lo, hi) * (k - a) + box_area(lo2, hi2) * (b - k);
        if (cost < best) { best = cost; best_k = k; }
      }
      run(a, best_k, parent_area);
      run(best_k, b, parent_area);
    }
    if (group) out[gi].skip = (int32_t)out.size();
  }
};

// The hierarchy over objects in the order `perm` (contiguous runs of finite-box objects).
static void build_hierarchy(FlatScene* fs, const std::vector<int>& perm, std::vector<RtTrav>* out) {
  HierBuilder h{*fs, *out, perm};
  out->clear();
  const int n = (int)perm.size();
  const bool flat = diag_env("RT_FLAT_OBJECTS");   // diagnostic: no group nodes
  for (int i = 0; i < n;) {
    if (flat || fs->objects[perm[i]].cull != RT_CULL_BOX) { h.object(i); ++i; continue; }
    int j = i;
    while (j < n && fs->objects[perm[j]].cull == RT_CULL_BOX) ++j;
    h.run(i, j, INFINITY);
    i = j;
  }
}

// Shadow rays of a scene without a transparent object only ask whether ANY object has a filtered
// hit in range (every transparency is +-0: the product is 0 at the first one), so their walk may
// visit the objects in any order and stop at the first occluder.  The likeliest occluders go
// first: objects by descending world volume of their region (the oriented box's where the object
// has one), unbounded objects (planes) last.  With a transparent object the draw order stays
// (the shadow product's order is the reference's).
static std::vector<int> shadow_order(const FlatScene& f) {
  const int n = (int)f.objects.size();
  std::vector<int> perm(n);
  for (int i = 0; i < n; ++i) perm[i] = i;
  if (f.any_transparent || diag_env("RT_DRAW_ORDER_SHADOWS")) return perm;
  std::vector<double> vol(n);
  for (int i = 0; i < n; ++i) {
    const RtObject& o = f.objects[i];
    if (o.cull != RT_CULL_BOX) { vol[i] = -1.0; continue; }          // unbounded: last
    double v = 1.0;
    for (int k = 0; k < 3; ++k) v *= o.bhi[k] - o.blo[k];
    if (o.obb_leaf >= 0) {
      const RtLeaf& R = f.leaves[o.obb_leaf];
      const double* M = R.inv;
      const double det = M[0] * (M[5] * M[10] - M[6] * M[9]) - M[1] * (M[4] * M[10] - M[6] * M[8]) +
                         M[2] * (M[4] * M[9] - M[5] * M[8]);
      double lv = 1.0;
      for (int k = 0; k < 3; ++k) lv *= o.ohi[k] - o.olo[k];
      if (std::isfinite(det) && det != 0.0) v = std::min(v, fabs(lv / det));
    }
    vol[i] = v;
  }
  std::stable_sort(perm.begin(), perm.end(), [&](int a, int b) { return vol[a] > vol[b]; });
  return perm;
}

// The flattened scene as text (rt_scene_describe): the flags, both hierarchies and every object's
// culling boxes, oriented box and leaf records -- what the kernels will read (tests, debugging).
std::string describe_flat(const FlatScene& f) {
  std::string s;
  char buf[1024];
  auto emit = [&](const char* fmt, auto... a) {
    snprintf(buf, sizeof buf, fmt, a...);
    s += buf;
  };
  emit("scene any_transparent=%d ray_chains=%d colour_fast=%d shadow_early_out=%d shadow_pow=%d\n",
          f.any_transparent, f.ray_chains, f.colour_fast, f.shadow_early_out, f.shadow_pow);
  for (size_t i = 0; i < f.trav.size(); ++i)
    emit("trav %zu obj=%d skip=%d box [%.3f %.3f %.3f]..[%.3f %.3f %.3f]\n", i, f.trav[i].obj, f.trav[i].skip,
            f.trav[i].blo[0], f.trav[i].blo[1], f.trav[i].blo[2], f.trav[i].bhi[0], f.trav[i].bhi[1], f.trav[i].bhi[2]);
  for (size_t i = 0; i < f.strav.size(); ++i)
    emit("strav %zu obj=%d skip=%d\n", i, f.strav[i].obj, f.strav[i].skip);
  for (size_t o = 0; o < f.objects.size(); ++o) {
    const RtObject& ob = f.objects[o];
    emit("object %zu cull=%d box [%.3f %.3f %.3f]..[%.3f %.3f %.3f] leaves %d leaf_cull=%d obb_leaf=%d "
            "[%.3f %.3f %.3f]..[%.3f %.3f %.3f]\n", o, ob.cull, ob.blo[0], ob.blo[1], ob.blo[2], ob.bhi[0], ob.bhi[1],
            ob.bhi[2], ob.leaf_count, ob.leaf_cull, ob.obb_leaf, ob.olo[0], ob.olo[1], ob.olo[2], ob.ohi[0], ob.ohi[1], ob.ohi[2]);
    for (int l = ob.leaf_begin; l < ob.leaf_begin + ob.leaf_count; ++l) {
      const RtLeaf& L = f.leaves[l];
      emit("   leaf %d kind=%d cull=%d box [%.3f %.3f %.3f]..[%.3f %.3f %.3f] prog %d lits %d (%d %d %d) const %d xdiag %d share %d axis %d\n", l, L.kind,
              L.cull, L.blo[0], L.blo[1], L.blo[2], L.bhi[0], L.bhi[1], L.bhi[2], L.prog_end - L.prog_begin, L.n_lit,
              L.n_lit > 0 ? L.lit[0] : -1, L.n_lit > 1 ? L.lit[1] : -1, L.n_lit > 2 ? L.lit[2] : -1, L.filter_const, L.xdiag, L.share_prev,
              L.plane_axis);
    }
  }
  return s;
}

// ---------------------------------------------------------------- f32 culling boxes
// The kernels' culling slab tests run in f32 (rt_device.h fbox_may_hit): every box is grown by
// RT_CULL32_MARGIN and rounded outward to f32, so the f32 box contains the f64 one plus a margin four
// times the rounding of any culled ray's origin (|o| <= RT_CULL32_COORD_MAX) to f32.  Boxes that are
// never tested (cull NONE / ALWAYS) get +-inf; the f64 boxes stay for the wavefront path.
static float f32_down(double x) {
  float v = (float)(x - RT_CULL32_MARGIN);
  if ((double)v > x - RT_CULL32_MARGIN) v = nextafterf(v, -INFINITY);
  return v;
}
static float f32_up(double x) {
  float v = (float)(x + RT_CULL32_MARGIN);
  if ((double)v < x + RT_CULL32_MARGIN) v = nextafterf(v, INFINITY);
  return v;
}
static void f32_box(const double* lo, const double* hi, bool tested, float* flo, float* fhi) {
  for (int i = 0; i < 3; ++i) {
    flo[i] = tested ? f32_down(lo[i]) : -INFINITY;
    fhi[i] = tested ? f32_up(hi[i]) : INFINITY;
  }
}
static void f32_boxes(FlatScene& f) {
  for (RtLeaf& L : f.leaves) f32_box(L.blo, L.bhi, L.cull == RT_CULL_BOX, L.fblo, L.fbhi);
  for (RtObject& o : f.objects) f32_box(o.olo, o.ohi, o.obb_leaf >= 0, o.folo, o.fohi);
  for (std::vector<RtTrav>* tv : {&f.trav, &f.strav})
    for (RtTrav& t : *tv) f32_box(t.blo, t.bhi, t.obj < 0 || t.cull == RT_CULL_BOX, t.fblo, t.fbhi);
}

int flatten(const rt_scene& s, FlatScene* out) {
  FlatScene& f = *out;
  f = FlatScene();
  f.width = (int32_t)s.width;
  f.height = (int32_t)s.height;
  f.max_depth = s.max_depth;
  f.any_transparent = 0;
  f.shadow_early_out = 1;
  // colour_fast: every operand of every colour op (color.rs:36-90) is finite and >= +0 (no NaN,
  // no -0, nothing negative), so the kernels' clamps may take the min/max form (rt_device.h
  // in_limit<FC>).  Sufficient: every solid material colour and light colour channel finite with
  // a clear sign bit, every reflectivity and transparency finite, sign bit clear, <= 1.  Then the
  // ambient term, the Lambert intensities (in [0, 1], 0 for NaN angles), the shadow products, the
  // weights 1 - w and w of every fold, and every clamped colour are all finite and >= +0.
  f.colour_fast = 1;
  // ray_chains: a hit spawns a refraction ray only if transparency != 0 and not TIR, a reflection
  // ray only if rp != 0 and (outside or TIR), rp = TIR ? refl + (1 - refl) * transp : refl
  // (raytracer.rs:242-267).  When every object has transparency == 0 or reflectivity == 0 (IEEE
  // comparisons: a NaN counts as nonzero), a refracted hit has rp = refl = +-0 (no reflection) and a
  // TIR hit has no refraction: every hit spawns at most one ray, so each pixel's rays form a chain.
  f.ray_chains = 1;
  // shadow_pow: a shadow ray's transparency is the product, in draw order, of the transparency of
  // every filtered hit in range, 0 at the first +-0 factor (raytracer.rs:181-197; objects of
  // transparency 1 are skipped).  When every other factor is ONE value T, the product is
  // fl(...fl(fl(1 * T) * T)...) over however many there are -- it depends on the count of T hits and
  // on whether a +-0 hit exists, not on their order -- so the wavefront pair path may evaluate
  // (shadow ray, object) pairs in any order and fold counts (k_wavefront.hip wfp_*).
  f.shadow_pow = 1;
  f.shadow_t = 0.0;
  bool have_t = false, any_zero = false;
  auto nonneg = [](double x) { return std::isfinite(x) && !std::signbit(x); };
  auto unit = [&](double x) { return nonneg(x) && x <= 1.0; };
  for (const ObjectRec& o : s.objects) {
    Flattener fl{s, f};
    fl.node_begin = (int32_t)f.nodes.size();
    RtObject ob;
    memset(&ob, 0, sizeof ob);
    ob.node_begin = fl.node_begin;
    ob.leaf_begin = (int32_t)f.leaves.size();
    int err = 0;
    fl.emit(o.shape, &err);
    if (err) return err;
    ob.node_count = (int32_t)f.nodes.size() - ob.node_begin;
    ob.leaf_count = (int32_t)f.leaves.size() - ob.leaf_begin;
    for (int32_t l = ob.leaf_begin; l < ob.leaf_begin + ob.leaf_count; ++l) f.leaves[l].object = (int32_t)f.objects.size();
    if (ob.node_count > 32) return fail(RT_ERR_UNSUPPORTED, "object with %d CSG nodes (max 32)", ob.node_count);
    // Hit-filter program per leaf: for every CSG ancestor, the sibling's is_inside test with
    // the polarity of csg.rs:43-95 (Union: !in, !in; Intersection: in, in; Difference: !in, in).
    Box obox = box_empty();
    int n_leaf_boxes_tighter = 0;
    for (int32_t ni = 0; ni < ob.node_count; ++ni) {
      const RtNode& n = f.nodes[ob.node_begin + ni];
      if (n.kind >= RT_N_UNION) continue;
      f.leaves[n.leaf].prog_begin = (int32_t)f.prog.size();
      Box useful = fl.box[ni];             // an accepted hit of this leaf lies on the leaf ...
      int32_t child = ni, par = fl.parent[ni];
      while (par >= 0) {
        const RtNode& P = f.nodes[ob.node_begin + par];
        bool is_a = P.a == child;
        int32_t sib = is_a ? P.b : P.a;
        int want = P.kind == RT_N_INTERSECTION ? 1 : P.kind == RT_N_UNION ? 0 : (is_a ? 0 : 1);
        fl.emit_inside(sib);
        f.prog.push_back({RT_OP_REQUIRE, want});
        if (want) useful = box_meet(useful, fl.box[sib]);   // ... and inside every required sibling
        child = par;
        par = fl.parent[par];
      }
      RtLeaf& L = f.leaves[n.leaf];
      L.prog_end = (int32_t)f.prog.size();
      L.n_lit = filter_literals(f.prog, L.prog_begin, L.prog_end, L.lit);
      L.cull = useful.kind;
      for (int i = 0; i < 3; ++i) { L.blo[i] = useful.lo[i]; L.bhi[i] = useful.hi[i]; }
      obox = box_hull(obox, useful);
    }
    ob.cull = obox.kind;
    for (int i = 0; i < 3; ++i) { ob.blo[i] = obox.lo[i]; ob.bhi[i] = obox.hi[i]; }
    // per-leaf box tests only pay when some leaf box is clearly tighter than the object's
    for (int32_t l = ob.leaf_begin; l < ob.leaf_begin + ob.leaf_count && ob.leaf_count > 1; ++l) {
      const RtLeaf& L = f.leaves[l];
      if (L.cull == RT_CULL_ALWAYS) ++n_leaf_boxes_tighter;
      else if (L.cull == RT_CULL_BOX && (ob.cull == RT_CULL_NONE || box_area(L.blo, L.bhi) < 0.8 * box_area(ob.blo, ob.bhi)))
        ++n_leaf_boxes_tighter;
    }
    ob.leaf_cull = n_leaf_boxes_tighter > 0;
    obb(f, &ob);
    unit_normal(f, &ob);
    order_literals(f, ob);
    const_filters(f, ob);
    const rt_material& m = o.mat;
    ob.textured = m.texture >= 0;
    ob.tex = m.texture >= 0 ? m.texture : 0;
    if (m.texture >= (int32_t)s.textures.size()) return fail(RT_ERR_INVALID, "bad texture id %d", m.texture);
    ob.color[0] = m.color[0]; ob.color[1] = m.color[1]; ob.color[2] = m.color[2]; ob.color_a = m.color[3];
    ob.reflectivity = m.reflectivity;
    ob.transparency = m.transparency;
    ob.shadow_skip = m.transparency == 1.0;
    if (m.transparency != 0.0) f.any_transparent = 1;
    if (m.transparency != 0.0 && m.reflectivity != 0.0) f.ray_chains = 0;
    if (!isfinite(m.transparency)) f.shadow_early_out = 0;
    if (m.transparency == 0.0) any_zero = true;
    if (m.transparency != 0.0 && m.transparency != 1.0) {
      if (!have_t) { f.shadow_t = m.transparency; have_t = true; }
      else if (memcmp(&f.shadow_t, &m.transparency, sizeof(double)) != 0) f.shadow_pow = 0;
    }
    if (!unit(m.reflectivity) || !unit(m.transparency)) f.colour_fast = 0;
    if (m.texture < 0 && !(nonneg(m.color[0]) && nonneg(m.color[1]) && nonneg(m.color[2]))) f.colour_fast = 0;
    f.objects.push_back(ob);
  }
  // The chain kernels' pool frames name their hit object in one byte (rt_device.h RT_POOL_OBJ_INDEX):
  // refraction scenes of more than 256 objects take the ray-tree kernels, which handle chains too.
  if (f.objects.size() > 256) f.ray_chains = 0;
  if (!f.shadow_early_out) f.shadow_pow = 0;
  // |T| > 1: T^k may overflow to +-inf, and inf * 0 is NaN, so with a zero-transparency object the
  // draw-order product depends on where the zero factor comes (T, T, 0 -> NaN; 0, T, T -> 0): not
  // a function of the counts
  if (have_t && !(fabs(f.shadow_t) <= 1.0) && any_zero) f.shadow_pow = 0;
  for (RtObject& ob : f.objects) share_sphere_terms(f, &ob);
  {
    std::vector<int> draw((size_t)f.objects.size());
    for (size_t i = 0; i < draw.size(); ++i) draw[i] = (int)i;
    build_hierarchy(&f, draw, &f.trav);
    build_hierarchy(&f, shadow_order(f), &f.strav);
  }
  f32_boxes(f);
  for (const LightRec& l : s.lights) {
    RtLight L;
    for (int i = 0; i < 3; ++i) { L.p[i] = l.p[i]; L.col[i] = l.color[i]; }
    if (!(nonneg(l.color[0]) && nonneg(l.color[1]) && nonneg(l.color[2]))) f.colour_fast = 0;
    f.lights.push_back(L);
  }
  int64_t off = 0;
  for (const TextureRec& t : s.textures) {
    RtTexture T;
    T.offset = off; T.w = (int32_t)t.w; T.h = (int32_t)t.h;
    f.textures.push_back(T);
    f.texels.insert(f.texels.end(), t.rgba.begin(), t.rgba.end());
    off += (int64_t)t.rgba.size();
    while (off % 16) { f.texels.push_back(0); ++off; }
  }
  // PerspectiveCamera::new(width, height, center, None, None, None) (camera.rs:30-54)
  V center = {s.cam_center[0], s.cam_center[1], s.cam_center[2]};
  V look_at = {0.0, 0.0, 0.0}, up = {0.0, 1.0, 0.0}, right = {0.0, 0.0, 0.0};
  V direction = normalized(sub(look_at, center));
  double aspect = (double)s.width / (double)s.height;
  if (length(right) == 0.0) { V c = cross(direction, up); right = {-c.x, -c.y, -c.z}; }
  RtCamera& cam = f.cam;
  cam.center[0] = center.x; cam.center[1] = center.y; cam.center[2] = center.z;
  cam.direction[0] = direction.x; cam.direction[1] = direction.y; cam.direction[2] = direction.z;
  cam.right[0] = right.x; cam.right[1] = right.y; cam.right[2] = right.z;
  cam.up[0] = up.x; cam.up[1] = up.y; cam.up[2] = up.z;
  cam.aspect = aspect;
  cam.width = (double)s.width;
  cam.height = (double)s.height;
  return RT_OK;
}

}  // namespace rt

using namespace rt;

// ==================================================================== C ABI: construction
extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }

int rt_xform_identity(rt_transformation* out) {
  if (!out) return fail(RT_ERR_INVALID, "null output");
  xf_identity(out);
  return RT_OK;
}
int rt_xform_translation(double x, double y, double z, rt_transformation* out) {
  if (!out) return fail(RT_ERR_INVALID, "null output");
  xf_translation(x, y, z, out);
  return RT_OK;
}
int rt_xform_rotation(double x, double y, double z, rt_transformation* out) {
  if (!out) return fail(RT_ERR_INVALID, "null output");
  xf_rotation(x, y, z, out);
  return RT_OK;
}
int rt_xform_scaling(double x, double y, double z, rt_transformation* out) {
  if (!out) return fail(RT_ERR_INVALID, "null output");
  xf_scaling(x, y, z, out);
  return RT_OK;
}
int rt_xform_compose(const rt_transformation* self_, const rt_transformation* other, rt_transformation* out) {
  if (!self_ || !other || !out) return fail(RT_ERR_INVALID, "null argument");
  xf_compose(*self_, *other, out);
  return RT_OK;
}

int rt_scene_new(uint32_t width, uint32_t height, rt_scene** out) {
  if (!out) return fail(RT_ERR_INVALID, "null output");
  *out = nullptr;
  if (width == 0 || height == 0 || width > 65536 || height > 65536)
    return fail(RT_ERR_INVALID, "bad frame size %ux%u", width, height);
  rt_scene* s = new (std::nothrow) rt_scene();
  if (!s) return fail(RT_ERR_NOMEM, "out of memory");
  s->width = width;
  s->height = height;
  *out = s;
  return RT_OK;
}

int rt_scene_traversal(const rt_scene* s, int32_t* obj, int32_t* skip, int32_t cap, int32_t* n) {
  if (!s || !n || cap < 0 || (cap > 0 && (!obj || !skip))) return fail(RT_ERR_INVALID, "null argument");
  FlatScene f;
  int rc = flatten(*s, &f);
  if (rc) return rc;
  *n = (int32_t)f.trav.size();
  for (int32_t i = 0; i < *n && i < cap; ++i) { obj[i] = f.trav[i].obj; skip[i] = f.trav[i].skip; }
  return RT_OK;
}

int rt_scene_describe(const rt_scene* s, char* buf, size_t cap, size_t* len) {
  if (!s || !len || (cap > 0 && !buf)) return fail(RT_ERR_INVALID, "null argument");
  FlatScene f;
  int rc = flatten(*s, &f);
  if (rc) return rc;
  const std::string d = describe_flat(f);
  *len = d.size();
  if (cap > 0) {
    const size_t n = d.size() < cap - 1 ? d.size() : cap - 1;
    memcpy(buf, d.data(), n);
    buf[n] = 0;
  }
  return RT_OK;
}

int rt_scene_add_test_objects(rt_scene* s) {                     // raytracer.rs:125-129
  if (!s) return fail(RT_ERR_INVALID, "null scene");
  LightRec l;
  l.p[0] = -10.0; l.p[1] = 30.0; l.p[2] = -50.0;
  l.color[0] = l.color[1] = l.color[2] = 0.5; l.color[3] = 1.0;   // Color::in_range(0.5, 0.5, 0.5)
  l.fade = 100.0;
  s->lights.push_back(l);
  return RT_OK;
}

int rt_scene_add_texture(rt_scene* s, uint32_t w, uint32_t h, const uint8_t* rgba8) {
  if (!s || !rgba8) return fail(RT_ERR_INVALID, "null argument");
  if (w == 0 || h == 0 || (uint64_t)w * h > (1ull << 28)) return fail(RT_ERR_INVALID, "bad texture size");
  TextureRec t;
  t.w = w; t.h = h;
  t.rgba.assign(rgba8, rgba8 + (size_t)w * h * 4);
  s->textures.push_back(std::move(t));
  return (int)s->textures.size() - 1;
}

static int add_shape(rt_scene* s, const ShapeRec& r) {
  s->shapes.push_back(r);
  return (int)s->shapes.size() - 1;
}

int rt_shape_sphere(rt_scene* s, const rt_transformation* t, const double c[3], double radius) {
  if (!s || !t || !c) return fail(RT_ERR_INVALID, "null argument");
  ShapeRec r;
  memset(&r, 0, sizeof r);
  r.kind = SHAPE_SPHERE; r.t = *t;
  memcpy(r.center, c, sizeof r.center);
  r.size = radius;
  return add_shape(s, r);
}
int rt_shape_cube(rt_scene* s, const rt_transformation* t, const double c[3], double length) {
  if (!s || !t || !c) return fail(RT_ERR_INVALID, "null argument");
  ShapeRec r;
  memset(&r, 0, sizeof r);
  r.kind = SHAPE_CUBE; r.t = *t;
  memcpy(r.center, c, sizeof r.center);
  r.size = length;
  return add_shape(s, r);
}
int rt_shape_plane(rt_scene* s, const rt_transformation* t, const double n[3], double distance) {
  if (!s || !t || !n) return fail(RT_ERR_INVALID, "null argument");
  ShapeRec r;
  memset(&r, 0, sizeof r);
  r.kind = SHAPE_PLANE; r.t = *t;
  memcpy(r.normal, n, sizeof r.normal);
  r.distance = distance;
  return add_shape(s, r);
}
int rt_shape_csg(rt_scene* s, rt_csg_op op, int32_t a, int32_t b) {
  if (!s) return fail(RT_ERR_INVALID, "null scene");
  if (a < 0 || b < 0 || a >= (int32_t)s->shapes.size() || b >= (int32_t)s->shapes.size())
    return fail(RT_ERR_INVALID, "bad CSG child id");
  if (op != RT_CSG_UNION && op != RT_CSG_INTERSECTION && op != RT_CSG_DIFFERENCE)
    return fail(RT_ERR_INVALID, "bad CSG operator %d", (int)op);
  ShapeRec r;
  memset(&r, 0, sizeof r);
  r.kind = SHAPE_CSG; r.op = op; r.a = a; r.b = b;
  xf_identity(&r.t);
  return add_shape(s, r);
}
int rt_scene_add_object(rt_scene* s, int32_t shape, const rt_material* m) {
  if (!s || !m) return fail(RT_ERR_INVALID, "null argument");
  if (shape < 0 || shape >= (int32_t)s->shapes.size()) return fail(RT_ERR_INVALID, "bad shape id %d", shape);
  if (m->texture >= (int32_t)s->textures.size()) return fail(RT_ERR_INVALID, "bad texture id %d", m->texture);
  s->objects.push_back({shape, *m});
  return RT_OK;
}
int rt_scene_add_light(rt_scene* s, const double p[3], const double col[4], double fade) {
  if (!s || !p || !col) return fail(RT_ERR_INVALID, "null argument");
  LightRec l;
  memcpy(l.p, p, sizeof l.p);
  memcpy(l.color, col, sizeof l.color);
  l.fade = fade;
  s->lights.push_back(l);
  return RT_OK;
}
int rt_scene_set_camera(rt_scene* s, const double c[3]) {
  if (!s || !c) return fail(RT_ERR_INVALID, "null argument");
  memcpy(s->cam_center, c, sizeof s->cam_center);
  return RT_OK;
}
int rt_scene_set_max_depth(rt_scene* s, int32_t d) {
  if (!s) return fail(RT_ERR_INVALID, "null scene");
  if (d < 0) return fail(RT_ERR_INVALID, "negative max_depth");
  if (d > RT_MAX_DEPTH_CAP) return fail(RT_ERR_UNSUPPORTED, "max_depth %d > %d", d, RT_MAX_DEPTH_CAP);
  s->max_depth = d;
  return RT_OK;
}
int rt_scene_info(const rt_scene* s, int32_t* n_objects, int32_t* n_lights, int32_t* n_leaves,
                  uint32_t* width, uint32_t* height) {
  if (!s) return fail(RT_ERR_INVALID, "null scene");
  if (n_objects) *n_objects = (int32_t)s->objects.size();
  if (n_lights) *n_lights = (int32_t)s->lights.size();
  if (n_leaves) {
    FlatScene f;
    int rc = flatten(*s, &f);
    if (rc) return rc;
    *n_leaves = (int32_t)f.leaves.size();
  }
  if (width) *width = s->width;
  if (height) *height = s->height;
  return RT_OK;
}
int rt_scene_get_camera(const rt_scene* s, double out[13]) {
  if (!s || !out) return fail(RT_ERR_INVALID, "null argument");
  FlatScene f;
  rt_scene tmp;                                       // camera only: no need to flatten objects
  tmp.width = s->width; tmp.height = s->height;
  memcpy(tmp.cam_center, s->cam_center, sizeof tmp.cam_center);
  int rc = flatten(tmp, &f);
  if (rc) return rc;
  for (int i = 0; i < 3; ++i) {
    out[i] = f.cam.center[i]; out[3 + i] = f.cam.direction[i]; out[6 + i] = f.cam.right[i]; out[9 + i] = f.cam.up[i];
  }
  out[12] = f.cam.aspect;
  return RT_OK;
}
int rt_scene_get_light(const rt_scene* s, int32_t i, double point[3], double color[4]) {
  if (!s || !point || !color) return fail(RT_ERR_INVALID, "null argument");
  if (i < 0 || i >= (int32_t)s->lights.size()) return fail(RT_ERR_INVALID, "light %d out of range", i);
  memcpy(point, s->lights[i].p, sizeof s->lights[i].p);
  memcpy(color, s->lights[i].color, sizeof s->lights[i].color);
  return RT_OK;
}
void rt_scene_free(rt_scene* s) { delete s; }

int rt_scene_compile(const char* text, const char* asset_dir, double time, uint32_t width,
                     uint32_t height, rt_scene** out) {
  if (!text || !out) return fail(RT_ERR_INVALID, "null argument");
  *out = nullptr;
  rt_scene* s = nullptr;
  int rc = rt_scene_new(width, height, &s);
  if (rc) return rc;
  rt_scene_add_test_objects(s);                                 // debug_window.rs:54-55
  rc = compile_scene_text(text, asset_dir, time, s);
  if (rc == RT_OK) { *out = s; return RT_OK; }
  if (rc == RT_ERR_PARSE) {                                     // default scene, error reported
    std::string msg = rt_last_error();
    rt_scene_free(s);
    rt_scene_new(width, height, &s);
    rt_scene_add_test_objects(s);
    *out = s;
    set_error_message(msg);
    return RT_ERR_PARSE;
  }
  rt_scene_free(s);
  return rc;
}

const char* rt_last_error(void) { return g_last_error.c_str(); }

}  // extern "C"
