/*
 * rt_oracle.c -- CPU ORACLE for the TinyRaytracer per-pixel render path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline.  The product (tinyraytracerinrust_amd/, librt_mi355x.so) never links,
 * loads or calls it; the product fails loudly when its HIP library is missing.
 *
 * What it is: a scalar f64 restatement, op for op, of the reference Rust code
 * (andreivasiliu/TinyRaytracerInRust, read-only at /root/reference), written in the
 * reference's own object model (shape "trait objects", CSG closures, recursive
 * get_ray_color) so that it is structurally independent of the product's flattened
 * GPU design.  Every function cites the reference file:line it restates.
 *
 * Parity status: UNPINNED by reference fixtures.  The reference ships no tests,
 * golden images or vectors and cannot be built here (no Rust
 * toolchain, crates not vendored).  The oracle is instead cross-checked bit-for-bit
 * (f64 colours) against an independent pure-Python restatement (oracle/pyref.py) on
 * small frames; see DESIGN.md "Oracle".
 *
 * Numerics: compiled with -O2 -ffp-contract=off, no fast-math; libm is glibc, the
 * same libm Rust's f64::{sin,cos,acos} call on Linux.  Sums are evaluated left to
 * right exactly as written in the Rust source.
 */
#define _GNU_SOURCE
#include <math.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#ifndef ORC_COUNTERS
#define ORC_COUNTERS 0
#endif

/* ------------------------------------------------------------------------- */
/* Event counters (compiled in only for the counting build).                  */
/* ------------------------------------------------------------------------- */
enum {
  C_RAY_PRIMARY, C_RAY_SHADOW, C_RAY_REFLECT, C_RAY_REFRACT,
  C_XFORM_RAY,          /* MatrixTransformation::reverse_transform_ray       */
  C_SPHERE_ISECT_MISS, C_SPHERE_ISECT_HIT,
  C_PLANE_ISECT, C_CUBE_ISECT_AXIS, C_CUBE_ISECT_ZERO_AXIS,
  C_CSG_POINT,          /* ray.point + ray.direction * d in a CSG closure     */
  C_INSIDE_SPHERE, C_INSIDE_CUBE, C_INSIDE_PLANE,
  C_ONSURF_SPHERE, C_ONSURF_CUBE, C_ONSURF_PLANE,
  C_NORMAL_SPHERE, C_NORMAL_CUBE_PLANECHK, C_NORMAL_PLANE,
  C_UV_SPHERE, C_TEXTURE_FETCH,
  C_SHADE,              /* shaded hits (point + normalize + ambient)          */
  C_LIGHT,              /* per-light shadow setup (dir, distance)             */
  C_LIGHT_LIT,          /* lights that pass the transparency test (angle etc.) */
  C_SHADOW_HIT,         /* transparency multiplications                       */
  C_INSIDE_TEST,        /* angle(-dir, n) per shaded hit                      */
  C_REFRACT_DIR, C_REFLECT_DIR, C_COMBINE,
  C_FLOP,               /* f64 add/sub/mul/div/sqrt + libm calls, as evaluated by the reference */
  C_TRANSC,             /* acos / sin calls (also inside C_FLOP)                               */
  C_NUM
};
#if ORC_COUNTERS
static __thread uint64_t *g_cnt;   /* NULL outside render jobs: scene setup is not counted */
#define CNT(e) (g_cnt ? (void)(g_cnt[(e)]++) : (void)0)
#define CNTN(e, n) (g_cnt ? (void)(g_cnt[(e)] += (uint64_t)(n)) : (void)0)
#else
#define CNT(e) ((void)0)
#define CNTN(e, n) ((void)0)
#endif
/* FL(n): n floating-point operations evaluated at this point of the reference code.  Negation,
 * comparisons, clamps and compile-time constants are not counted; sqrt, division and each libm
 * call count 1 (transcendentals are also tallied in C_TRANSC). */
#define FL(n) CNTN(C_FLOP, (n))
#define TR(n) (CNTN(C_FLOP, (n)), CNTN(C_TRANSC, (n)))

/* ------------------------------------------------------------------------- */
/* math.rs:1-24, vector.rs:3-120                                              */
/* ------------------------------------------------------------------------- */
static const double EPSILON = 10e-7;          /* math.rs:2 (== 1e-6) */
static const double PI = 3.14159265358979323846; /* std::f64::consts::PI */

typedef struct { double x, y, z; } Vec;
typedef struct { Vec point, direction; } Ray;
typedef struct { double u, v; } UV;

static Vec v_new(double x, double y, double z) { Vec r = {x, y, z}; return r; }
static Vec v_add(Vec a, Vec b) { FL(3); return v_new(a.x + b.x, a.y + b.y, a.z + b.z); }   /* vector.rs:70-80 */
static Vec v_sub(Vec a, Vec b) { FL(3); return v_new(a.x - b.x, a.y - b.y, a.z - b.z); }   /* vector.rs:82-92 */
static double v_dot(Vec a, Vec b) { FL(5); return a.x * b.x + a.y * b.y + a.z * b.z; }     /* vector.rs:94-100 */
static Vec v_scale(Vec a, double s) { FL(3); return v_new(a.x * s, a.y * s, a.z * s); }    /* vector.rs:102-112 */
static Vec v_neg(Vec a) { return v_new(-a.x, -a.y, -a.z); }                         /* vector.rs:114-120 */
static double v_length(Vec a) { FL(1); return sqrt(v_dot(a, a)); }                         /* vector.rs:49-51 */
static Vec v_normalized(Vec a) { FL(1); return v_scale(a, 1.0 / v_length(a)); }            /* vector.rs:45-47 */
static double v_angle(Vec a, Vec b) {                                               /* vector.rs:57-59 */
  FL(2); TR(1);
  return acos(v_dot(a, b) / (v_length(a) * v_length(b)));
}
static Vec v_cross(Vec a, Vec b) {                                                  /* vector.rs:61-67 */
  FL(9);
  return v_new(a.y * b.z - a.z * b.y, a.x * b.z - a.z * b.x, a.x * b.y - a.y * b.x);
}

/* ------------------------------------------------------------------------- */
/* color.rs:1-90                                                              */
/* ------------------------------------------------------------------------- */
typedef struct { double r, g, b, a; } Color;
static const Color BLACK = {0.0, 0.0, 0.0, 1.0};

static double in_limit(double x, double mn, double mx) {                            /* color.rs:36-44 */
  if (x < mn) return mn;
  else if (x > mx) return mx;
  else return x;
}
static Color in_range(double r, double g, double b) {                              /* color.rs:46-53 */
  Color c = {in_limit(r, 0.0, 1.0), in_limit(g, 0.0, 1.0), in_limit(b, 0.0, 1.0), 1.0};
  return c;
}
static Color c_intensify(Color c, double k) { FL(3); return in_range(c.r * k, c.g * k, c.b * k); } /* color.rs:71-73 */
static Color c_mul(Color a, Color b) { FL(3); return in_range(a.r * b.r, a.g * b.g, a.b * b.b); }  /* color.rs:76-82 */
static Color c_add(Color a, Color b) { FL(3); return in_range(a.r + b.r, a.g + b.g, a.b + b.b); }  /* color.rs:84-90 */

/* Rust `(x * 255.0) as u8`: saturating, truncating, NaN -> 0 (easy_pixbuf.rs:49-52). */
static uint8_t to_u8(double c) {
  double v = c * 255.0;
  if (!(v > 0.0)) return 0;          /* NaN, negative, zero */
  if (v >= 255.0) return 255;
  return (uint8_t)v;
}

/* ------------------------------------------------------------------------- */
/* transformation.rs:47-220                                                   */
/* ------------------------------------------------------------------------- */
typedef struct { double m[4][4]; double inv[4][4]; } Xform;

static Vec transform_vector(Vec v, const double m[4][4]) {                          /* transformation.rs:53-59 */
  FL(18);
  double a = m[0][0] * v.x + m[0][1] * v.y + m[0][2] * v.z + m[0][3];
  double b = m[1][0] * v.x + m[1][1] * v.y + m[1][2] * v.z + m[1][3];
  double c = m[2][0] * v.x + m[2][1] * v.y + m[2][2] * v.z + m[2][3];
  return v_new(a, b, c);
}
static Vec xf_transform_vector(const Xform *t, Vec v) { return transform_vector(v, t->m); }        /* :62-64 */
static Vec xf_reverse_transform_vector(const Xform *t, Vec v) { return transform_vector(v, t->inv); } /* :66-68 */
static Vec xf_transform_direction_vector(const Xform *t, Vec v) {                   /* :70-77 */
  Vec o = transform_vector(v_new(0.0, 0.0, 0.0), t->m);
  return v_sub(transform_vector(v, t->m), o);
}
static Vec xf_reverse_transform_direction_vector(const Xform *t, Vec v) {           /* :79-86 */
  Vec o = transform_vector(v_new(0.0, 0.0, 0.0), t->inv);
  return v_sub(transform_vector(v, t->inv), o);
}
static Ray xf_reverse_transform_ray(const Xform *t, Ray r) {                        /* :88-93 */
  Ray o;
  CNT(C_XFORM_RAY);
  o.point = xf_reverse_transform_vector(t, r.point);
  o.direction = xf_reverse_transform_direction_vector(t, r.direction);
  return o;
}
static void multiply_matrices(const double a[4][4], const double b[4][4], double out[4][4]) { /* :208-220 */
  double res[4][4];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      res[i][j] = 0.0;                       /* Default::default() */
      for (int k = 0; k < 4; ++k) res[i][j] += a[i][k] * b[k][j];
    }
  memcpy(out, res, sizeof res);
}
static Xform xf_identity(void) {                                                    /* :104-113 */
  Xform t;
  memset(&t, 0, sizeof t);
  for (int i = 0; i < 4; ++i) t.m[i][i] = t.inv[i][i] = 1.0;
  return t;
}
static void rot_x(double a, double m[4][4]) {                                       /* :116-125 */
  double c = cos(a), s = sin(a);
  double r[4][4] = {{1, 0, 0, 0}, {0, c, -s, 0}, {0, s, c, 0}, {0, 0, 0, 1}};
  memcpy(m, r, sizeof r);
}
static void rot_y(double a, double m[4][4]) {                                       /* :127-136 */
  double c = cos(a), s = sin(a);
  double r[4][4] = {{c, 0, -s, 0}, {0, 1, 0, 0}, {s, 0, c, 0}, {0, 0, 0, 1}};
  memcpy(m, r, sizeof r);
}
static void rot_z(double a, double m[4][4]) {                                       /* :138-147 */
  double c = cos(a), s = sin(a);
  double r[4][4] = {{c, -s, 0, 0}, {s, c, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
  memcpy(m, r, sizeof r);
}
static Xform xf_rotation(double x, double y, double z) {                            /* :115-162 */
  double m1[4][4], i1[4][4], m2[4][4], i2[4][4], m3[4][4], i3[4][4], tmp[4][4];
  Xform t;
  rot_x(x, m1); rot_x(-x, i1);
  rot_y(y, m2); rot_y(-y, i2);
  rot_z(z, m3); rot_z(-z, i3);
  multiply_matrices(m1, m2, tmp); multiply_matrices(tmp, m3, t.m);
  multiply_matrices(i1, i2, tmp); multiply_matrices(tmp, i3, t.inv);
  return t;
}
static Xform xf_translation(double x, double y, double z) {                         /* :164-180 */
  Xform t = xf_identity();
  t.m[0][3] = x; t.m[1][3] = y; t.m[2][3] = z;
  t.inv[0][3] = -x; t.inv[1][3] = -y; t.inv[2][3] = -z;
  return t;
}
static Xform xf_scaling(double x, double y, double z) {                             /* :182-198 */
  Xform t = xf_identity();
  t.m[0][0] = x; t.m[1][1] = y; t.m[2][2] = z;
  t.inv[0][0] = 1.0 / x; t.inv[1][1] = 1.0 / y; t.inv[2][2] = 1.0 / z;
  return t;
}
static Xform xf_compose_with(const Xform *self, const Xform *other) {               /* :200-205 */
  Xform t;
  multiply_matrices(other->m, self->m, t.m);
  multiply_matrices(self->inv, other->inv, t.inv);
  return t;
}

/* ------------------------------------------------------------------------- */
/* Textures: texture.rs:27-34 (lookup), sceneparser/texture.rs:20-40 (decode)  */
/* ------------------------------------------------------------------------- */
typedef struct Texture {
  char name[256];
  int w, h;
  Color *pix;  /* f64 RGBA pixmap, row-major, /255.0 exactly as sceneparser/texture.rs:29-33 */
  struct Texture *next;
} Texture;
static Texture *g_textures;
static pthread_mutex_t g_tex_lock = PTHREAD_MUTEX_INITIALIZER;

int orc_register_texture(const char *name, int w, int h, const uint8_t *rgba8) {
  Texture *t = (Texture *)calloc(1, sizeof *t);
  if (!t || w <= 0 || h <= 0) return -1;
  snprintf(t->name, sizeof t->name, "%s", name);
  t->w = w; t->h = h;
  t->pix = (Color *)malloc(sizeof(Color) * (size_t)w * (size_t)h);
  for (size_t i = 0; i < (size_t)w * (size_t)h; ++i) {
    t->pix[i].r = rgba8[4 * i + 0] / 255.0;
    t->pix[i].g = rgba8[4 * i + 1] / 255.0;
    t->pix[i].b = rgba8[4 * i + 2] / 255.0;
    t->pix[i].a = rgba8[4 * i + 3] / 255.0;
  }
  pthread_mutex_lock(&g_tex_lock);
  t->next = g_textures; g_textures = t;
  pthread_mutex_unlock(&g_tex_lock);
  return 0;
}
static Texture *find_texture(const char *name) {
  pthread_mutex_lock(&g_tex_lock);
  Texture *t = g_textures;
  while (t && strcmp(t->name, name) != 0) t = t->next;
  pthread_mutex_unlock(&g_tex_lock);
  return t;
}
/* Rust `f64 as usize`: saturating, NaN -> 0. */
static size_t f2usize(double v) {
  if (!(v > 0.0)) return 0;
  if (v >= 18446744073709551615.0) return (size_t)-1;
  return (size_t)v;
}
static Color texture_color_at(const Texture *t, UV uv) {                           /* texture.rs:27-34 */
  double x = uv.u * (double)(t->w - 1);
  double y = (double)t->h - (uv.v * (double)(t->h - 1)) - 1.0;
  FL(4);
  size_t xi = f2usize(x), yi = f2usize(y);
  CNT(C_TEXTURE_FETCH);
  /* The reference would panic on an out-of-bounds index; clamp instead. */
  if (xi >= (size_t)t->w) xi = (size_t)t->w - 1;
  if (yi >= (size_t)t->h) yi = (size_t)t->h - 1;
  return t->pix[yi * (size_t)t->w + xi];
}

/* ------------------------------------------------------------------------- */
/* Materials: material.rs:5-102                                               */
/* ------------------------------------------------------------------------- */
typedef struct {
  int textured;            /* 0: SolidColorMaterial, 1: TexturedMaterial */
  Color color;
  const Texture *texture;
  double reflectivity, transparency;
} Material;

static Color mat_color_at(const Material *m, UV uv) {                               /* material.rs:52-54, 87-89 */
  return m->textured ? texture_color_at(m->texture, uv) : m->color;
}

/* ------------------------------------------------------------------------- */
/* Shapes: math_shapes.rs, csg.rs, rt_object.rs                               */
/* ------------------------------------------------------------------------- */
typedef void (*AddIntersection)(void *ctx, double d);   /* math_shapes.rs:5 */

typedef enum { SH_SPHERE, SH_PLANE, SH_CUBE, SH_CSG } ShKind;
typedef enum { OP_UNION, OP_INTERSECTION, OP_DIFFERENCE } CsgOp;

typedef struct Plane { Xform t; double a, b, c, d; Vec normal; } Plane;
struct RTObject;
typedef struct Shape {
  ShKind kind;
  Xform t;
  /* sphere */ Vec center; double radius;
  /* plane  */ Plane plane;
  /* cube   */ Plane p1, p2, p3, p4, p5, p6; double length;
  /* csg    */ struct RTObject *a_obj, *b_obj; CsgOp op;
} Shape;
typedef struct RTObject { Shape *shape; Material material; } RTObject;

static Plane plane_new(Xform t, double a, double b, double c, double d) {           /* math_shapes.rs:140-152 */
  Plane p;
  p.t = t; p.a = a; p.b = b; p.c = c; p.d = d;
  Vec n = v_normalized(v_new(a, b, c));
  p.normal = v_normalized(xf_transform_direction_vector(&t, n));                   /* :158-160 */
  return p;
}
static int plane_is_transformed_point_on_surface(const Plane *p, Vec q) {           /* :162-164 */
  FL(6);
  return fabs(p->a * q.x + p->b * q.y + p->c * q.z + p->d) < EPSILON;
}

static void shape_intersects(const Shape *s, Ray ray, AddIntersection add, void *ctx);
static Vec shape_get_normal(const Shape *s, Vec p);
static int shape_is_inside(const Shape *s, Vec p);
static int shape_is_on_surface(const Shape *s, Vec p);
static int shape_get_uv(const Shape *s, Vec p, UV *out);

static Ray shape_reverse_transform_ray(const Shape *s, Ray r) {                     /* math_shapes.rs:17-19, csg.rs:178-181 */
  if (s->kind == SH_CSG) return r;
  return xf_reverse_transform_ray(&s->t, r);
}
static void rtobject_intersects(const RTObject *o, Ray ray, AddIntersection add, void *ctx) { /* rt_object.rs:28-31 */
  Ray tr = shape_reverse_transform_ray(o->shape, ray);
  shape_intersects(o->shape, tr, add, ctx);
}

/* --- MathSphere (math_shapes.rs:28-127) --- */
static void sphere_intersects(const Shape *s, Ray ray, AddIntersection add, void *ctx) { /* :42-62 */
  Vec v = v_sub(ray.point, s->center);
  Vec d = v_normalized(ray.direction);
  double scale = 1.0 / v_length(ray.direction);
  double r = s->radius;
  FL(5);
  double vd = v_dot(v, d);
  double sum = vd * vd - (v_dot(v, v) - r * r);
  if (sum < 0.0) { CNT(C_SPHERE_ISECT_MISS); return; }
  CNT(C_SPHERE_ISECT_HIT);
  FL(6);
  double first = (-vd + sqrt(sum)) * scale;
  double second = (-vd - sqrt(sum)) * scale;
  add(ctx, first);
  add(ctx, second);
}
static Vec sphere_get_normal(const Shape *s, Vec p) {                               /* :64-68 */
  CNT(C_NORMAL_SPHERE);
  Vec q = xf_reverse_transform_vector(&s->t, p);
  Vec n = v_sub(q, s->center);
  return v_normalized(xf_transform_direction_vector(&s->t, n));
}
static int sphere_is_inside(const Shape *s, Vec p) {                                /* :70-74 */
  CNT(C_INSIDE_SPHERE);
  Vec q = xf_reverse_transform_vector(&s->t, p);
  FL(1);
  return v_length(v_sub(q, s->center)) <= s->radius + EPSILON;
}
static int sphere_is_on_surface(const Shape *s, Vec p) {                            /* :76-80 */
  CNT(C_ONSURF_SPHERE);
  Vec q = xf_reverse_transform_vector(&s->t, p);
  FL(1);
  return fabs(v_length(v_sub(q, s->center)) - s->radius) < EPSILON;
}
static UV sphere_get_uv(const Shape *s, Vec p) {                                    /* :82-114 */
  CNT(C_UV_SPHERE);
  Vec q = xf_reverse_transform_vector(&s->t, v_sub(p, s->center));
  q = v_scale(v_normalized(q), 1.0 - EPSILON);
  Vec up = v_new(0.0, 1.0, 0.0);
  Vec u_zero = v_new(0.0, 0.0, -1.0);
  Vec u_qrtr = v_new(-1.0, 0.0, 0.0);
  TR(1);
  double phi = acos(-(v_dot(up, q)));
  if (isnan(phi)) phi = 0.0;   /* eprintln! + 0.0 (:91-96) */
  TR(2); FL(3);
  double theta = (acos(v_dot(q, u_zero) / sin(phi))) / (2.0 * PI);
  if (isnan(theta)) theta = 0.0;
  double v = phi / PI;
  double u = (v_dot(u_qrtr, q) > 0.0) ? (FL(1), 1.0 - theta) : theta;
  UV uv = {u, v};
  return uv;
}

/* --- MathPlane (math_shapes.rs:129-212) --- */
static void plane_intersects(const Plane *p, Ray ray, AddIntersection add, void *ctx) { /* :168-180 */
  CNT(C_PLANE_ISECT);
  Vec p_n = v_normalized(v_new(p->a, p->b, p->c));
  Vec r_0 = ray.point, r_d = ray.direction;
  double v_d = v_dot(p_n, r_d);
  if (v_d != 0.0) {
    FL(3);
    double t = -(v_dot(p_n, r_0) + p->d) * (1.0 / v_d);
    if (t >= 0.0) add(ctx, t);
  }
}
static int plane_is_on_surface(const Plane *p, Vec q) {                             /* :190-194 */
  CNT(C_ONSURF_PLANE);
  return plane_is_transformed_point_on_surface(p, xf_reverse_transform_vector(&p->t, q));
}

/* --- MathCube (math_shapes.rs:214-379) --- */
static void cube_init(Shape *s, Xform t, Vec center, double length) {               /* :228-244 */
  length = length / 2.0;
  s->p1 = plane_new(t, 0.0, 0.0, 1.0, -(center.z + length / 2.0));
  s->p6 = plane_new(t, 0.0, 0.0, -1.0, center.z + -length / 2.0);
  s->p2 = plane_new(t, 0.0, 1.0, 0.0, -(center.y + length / 2.0));
  s->p5 = plane_new(t, 0.0, -1.0, 0.0, center.y + -length / 2.0);
  s->p3 = plane_new(t, 1.0, 0.0, 0.0, -(center.x + length / 2.0));
  s->p4 = plane_new(t, -1.0, 0.0, 0.0, center.x + -length / 2.0);
  s->t = t; s->center = center; s->length = length;
}
static void cube_intersects(const Shape *s, Ray ray, AddIntersection add, void *ctx) { /* :248-290 */
  double t_near = -INFINITY, t_far = INFINITY;
  double dv[3] = {ray.direction.x, ray.direction.y, ray.direction.z};
  double pv[3] = {ray.point.x, ray.point.y, ray.point.z};
  double cv[3] = {s->center.x, s->center.y, s->center.z};
  for (int i = 0; i < 3; ++i) {
    if (dv[i] == 0.0) {
      CNT(C_CUBE_ISECT_ZERO_AXIS);
      FL(1);
      if (!(pv[i] < cv[i] - s->length)) FL(1);
      if (pv[i] < cv[i] - s->length || pv[i] > cv[i] + s->length) return;
      continue;
    }
    CNT(C_CUBE_ISECT_AXIS);
    FL(6);
    double t1 = (cv[i] - s->length - pv[i]) / dv[i];
    double t2 = (cv[i] + s->length - pv[i]) / dv[i];
    if (t1 > t2) { double tmp = t1; t1 = t2; t2 = tmp; }
    if (t1 > t_near) t_near = t1;
    if (t2 < t_far) t_far = t2;
    if (t_near > t_far || t_far < 0.0) return;
  }
  add(ctx, t_near);
  add(ctx, t_far);
}
static Vec cube_get_normal(const Shape *s, Vec p) {                                 /* :292-317 */
  Vec q = xf_reverse_transform_vector(&s->t, p);
  const Plane *planes[6] = {&s->p1, &s->p2, &s->p3, &s->p4, &s->p5, &s->p6};
  for (int i = 0; i < 6; ++i) {
    CNT(C_NORMAL_CUBE_PLANECHK);
    if (plane_is_transformed_point_on_surface(planes[i], q)) return planes[i]->normal;
  }
  return v_new(1.0, 1.0, 1.0);
}
static int cube_is_inside(const Shape *s, Vec p) {                                  /* :319-328 */
  CNT(C_INSIDE_CUBE);
  Vec q = xf_reverse_transform_vector(&s->t, p);
  FL(6);
  return q.x <= (s->center.x + s->length) && q.x >= (s->center.x - s->length) &&
         q.y <= (s->center.y + s->length) && q.y >= (s->center.y - s->length) &&
         q.z <= (s->center.z + s->length) && q.z >= (s->center.z - s->length);
}
static int is_between(double x, double start, double end) { return start <= x && x <= end; }
/* the bound expressions `c - l - EPSILON` / `c + l + EPSILON` are 4 flops per is_between */
#define BETWEEN(x, lo, hi) (FL(4), is_between((x), (lo), (hi))) /* :333-335 */
static int cube_is_on_surface(const Shape *s, Vec p) {                              /* :330-355 */
  CNT(C_ONSURF_CUBE);
  Vec q = xf_reverse_transform_vector(&s->t, p);
  Vec c = s->center;
  double l = s->length;
  if (BETWEEN(q.y, c.y - l - EPSILON, c.y + l + EPSILON) &&
      BETWEEN(q.x, c.x - l - EPSILON, c.x + l + EPSILON) &&
      (plane_is_transformed_point_on_surface(&s->p1, q) || plane_is_transformed_point_on_surface(&s->p6, q)))
    return 1;
  else if (BETWEEN(q.z, c.z - l - EPSILON, c.z + l + EPSILON) &&
           BETWEEN(q.x, c.x - l - EPSILON, c.x + l + EPSILON) &&
           (plane_is_transformed_point_on_surface(&s->p2, q) || plane_is_transformed_point_on_surface(&s->p5, q)))
    return 1;
  else if (BETWEEN(q.y, c.y - l - EPSILON, c.y + l + EPSILON) &&
           BETWEEN(q.z, c.z - l - EPSILON, c.z + l + EPSILON) &&
           (plane_is_transformed_point_on_surface(&s->p3, q) || plane_is_transformed_point_on_surface(&s->p4, q)))
    return 1;
  return 0;
}

/* --- CSG (csg.rs:38-186) --- */
typedef struct {
  const Shape *other;   /* the sibling whose is_inside filters the hit */
  int want_inside;      /* 1: keep if other.is_inside, 0: keep if !other.is_inside */
  Ray ray;
  AddIntersection add;
  void *ctx;
} CsgFilter;
static void csg_check(void *vctx, double d) {                                       /* csg.rs:45-49 etc. */
  CsgFilter *f = (CsgFilter *)vctx;
  CNT(C_CSG_POINT);
  Vec p = v_add(f->ray.point, v_scale(f->ray.direction, d));
  int in = shape_is_inside(f->other, p);
  if (f->want_inside ? in : !in) f->add(f->ctx, d);
}
static void csg_intersects(const Shape *s, Ray ray, AddIntersection add, void *ctx) { /* csg.rs:39-96 */
  const Shape *a = s->a_obj->shape, *b = s->b_obj->shape;
  CsgFilter fa = {b, 0, ray, add, ctx}, fb = {a, 0, ray, add, ctx};
  switch (s->op) {
    case OP_UNION:        fa.want_inside = 0; fb.want_inside = 0; break;
    case OP_INTERSECTION: fa.want_inside = 1; fb.want_inside = 1; break;
    case OP_DIFFERENCE:   fa.want_inside = 0; fb.want_inside = 1; break;
  }
  rtobject_intersects(s->a_obj, ray, csg_check, &fa);
  rtobject_intersects(s->b_obj, ray, csg_check, &fb);
}
static Vec csg_get_normal(const Shape *s, Vec p) {                                  /* csg.rs:98-124 */
  const Shape *a = s->a_obj->shape, *b = s->b_obj->shape;
  if (s->op == OP_DIFFERENCE) {
    if (shape_is_on_surface(a, p)) return shape_get_normal(a, p);
    else if (shape_is_on_surface(b, p)) return v_scale(shape_get_normal(b, p), -1.0);
    return v_new(1.0, 0.0, 0.0);
  }
  if (shape_is_on_surface(a, p)) return shape_get_normal(a, p);
  else if (shape_is_on_surface(b, p)) return shape_get_normal(b, p);
  return v_new(1.0, 0.0, 0.0);
}
static int csg_is_inside(const Shape *s, Vec p) {                                   /* csg.rs:126-135 */
  const Shape *a = s->a_obj->shape, *b = s->b_obj->shape;
  switch (s->op) {
    case OP_UNION: return shape_is_inside(a, p) || shape_is_inside(b, p);
    case OP_INTERSECTION: return shape_is_inside(a, p) && shape_is_inside(b, p);
    default: return shape_is_inside(a, p) && !shape_is_inside(b, p);
  }
}
static int csg_is_on_surface(const Shape *s, Vec p) {                               /* csg.rs:137-155 */
  const Shape *a = s->a_obj->shape, *b = s->b_obj->shape;
  switch (s->op) {
    case OP_UNION:
      return (shape_is_on_surface(a, p) && !shape_is_inside(b, p)) ||
             (shape_is_on_surface(b, p) && !shape_is_inside(a, p));
    case OP_INTERSECTION:
      return (shape_is_on_surface(a, p) && shape_is_inside(b, p)) ||
             (shape_is_on_surface(b, p) && shape_is_inside(a, p));
    default:
      return (shape_is_on_surface(a, p) && !shape_is_inside(b, p)) ||
             (shape_is_on_surface(b, p) && shape_is_inside(a, p));
  }
}
static int csg_get_uv(const Shape *s, Vec p, UV *out) {                             /* csg.rs:157-168 */
  const Shape *a = s->a_obj->shape, *b = s->b_obj->shape;
  if (shape_is_on_surface(a, p)) return shape_get_uv(a, p, out);
  else if (shape_is_on_surface(b, p)) return shape_get_uv(b, p, out);
  return 0;
}

/* --- dynamic dispatch (the `dyn MathShape` vtable) --- */
static void shape_intersects(const Shape *s, Ray ray, AddIntersection add, void *ctx) {
  switch (s->kind) {
    case SH_SPHERE: sphere_intersects(s, ray, add, ctx); break;
    case SH_PLANE: plane_intersects(&s->plane, ray, add, ctx); break;
    case SH_CUBE: cube_intersects(s, ray, add, ctx); break;
    case SH_CSG: csg_intersects(s, ray, add, ctx); break;
  }
}
static Vec shape_get_normal(const Shape *s, Vec p) {
  switch (s->kind) {
    case SH_SPHERE: return sphere_get_normal(s, p);
    case SH_PLANE: CNT(C_NORMAL_PLANE); return s->plane.normal;                   /* math_shapes.rs:182-184 */
    case SH_CUBE: return cube_get_normal(s, p);
    default: return csg_get_normal(s, p);
  }
}
static int shape_is_inside(const Shape *s, Vec p) {
  switch (s->kind) {
    case SH_SPHERE: return sphere_is_inside(s, p);
    case SH_PLANE: CNT(C_INSIDE_PLANE); return 0;                                 /* math_shapes.rs:186-188 */
    case SH_CUBE: return cube_is_inside(s, p);
    default: return csg_is_inside(s, p);
  }
}
static int shape_is_on_surface(const Shape *s, Vec p) {
  switch (s->kind) {
    case SH_SPHERE: return sphere_is_on_surface(s, p);
    case SH_PLANE: return plane_is_on_surface(&s->plane, p);
    case SH_CUBE: return cube_is_on_surface(s, p);
    default: return csg_is_on_surface(s, p);
  }
}
static int shape_get_uv(const Shape *s, Vec p, UV *out) {
  switch (s->kind) {
    case SH_SPHERE: *out = sphere_get_uv(s, p); return 1;
    case SH_PLANE: return 0;   /* Err("UV not implemented for MathPlane!") */
    case SH_CUBE: return 0;    /* Err("UV not implemented for MathCube!") */
    default: return csg_get_uv(s, p, out);
  }
}

/* ------------------------------------------------------------------------- */
/* Camera (camera.rs:17-79) and RayTracer (raytracer.rs:21-364)               */
/* ------------------------------------------------------------------------- */
typedef struct {
  int width, height;
  Vec center, look_at, up, right, direction;
  double aspect_ratio;
} Camera;

static Camera camera_new(int width, int height, Vec center) {                       /* camera.rs:30-54 */
  Camera c;
  c.width = width; c.height = height; c.center = center;
  c.look_at = v_new(0.0, 0.0, 0.0);
  c.up = v_new(0.0, 1.0, 0.0);
  Vec right = v_new(0.0, 0.0, 0.0);
  c.direction = v_normalized(v_sub(c.look_at, center));
  c.aspect_ratio = (double)width / (double)height;
  if (v_length(right) == 0.0) right = v_neg(v_cross(c.direction, c.up));
  c.right = right;
  return c;
}
static Ray camera_create_ray(const Camera *c, double x, double y) {                 /* camera.rs:65-74 */
  FL(7);
  double sx = ((x / (double)c->width) - 0.5) * c->aspect_ratio;
  double sy = ((double)c->height - 1.0 - y) / (double)c->height - 0.5;
  Ray r;
  r.direction = v_add(v_add(c->direction, v_scale(c->right, sx)), v_scale(c->up, sy));
  r.point = c->center;
  return r;
}

typedef struct { Vec point; Color color; double fade_distance; } PointLight;       /* point_light.rs:4-18 */

typedef struct Arena { struct Arena *next; size_t used, cap; char data[]; } Arena;

typedef struct orc_scene {
  int width, height, max_depth;
  Camera camera;
  RTObject *objects; int n_objects, cap_objects;
  PointLight *lights; int n_lights, cap_lights;
  Xform *xstack; int n_x, cap_x;     /* TransformationStack (transformation.rs:7-37) */
  Arena *arena;
} orc_scene;

static void *arena_alloc(orc_scene *sc, size_t n) {
  n = (n + 15) & ~(size_t)15;
  if (!sc->arena || sc->arena->used + n > sc->arena->cap) {
    size_t cap = n > 65536 ? n : 65536;
    Arena *a = (Arena *)malloc(sizeof(Arena) + cap);
    a->next = sc->arena; a->used = 0; a->cap = cap;
    sc->arena = a;
  }
  void *p = sc->arena->data + sc->arena->used;
  sc->arena->used += n;
  memset(p, 0, n);
  return p;
}

/* Nearest-hit closure state (raytracer.rs:138-150). */
typedef struct { double nearest; const RTObject *nearest_obj; const RTObject *cur; } NearestCtx;
static void add_nearest(void *vctx, double d) {                                     /* raytracer.rs:142-147 */
  NearestCtx *c = (NearestCtx *)vctx;
  if (d > EPSILON && d < c->nearest) { c->nearest = d; c->nearest_obj = c->cur; }
}
/* Shadow closure state (raytracer.rs:181-197). */
typedef struct { double distance; double transparency; const RTObject *cached; UV uv; } ShadowCtx;
static void add_shadow(void *vctx, double d) {                                      /* raytracer.rs:187-192 */
  ShadowCtx *c = (ShadowCtx *)vctx;
  if (d > EPSILON && d < c->distance) {
    CNT(C_SHADOW_HIT);
    FL(1);
    c->transparency *= c->cached->material.transparency;   /* get_transparency_at_uv(uv): constant */
  }
}

static Vec reflected_dir(Vec incident, Vec normal) {                                /* raytracer.rs:332-334 */
  CNT(C_REFLECT_DIR);
  return v_sub(incident, v_scale(v_scale(normal, 2.0), v_dot(normal, incident)));
}
static Vec refracted_dir(Vec incident, Vec normal, double r, int *tir) {            /* raytracer.rs:336-353 */
  CNT(C_REFRACT_DIR);
  double cos_1 = v_dot(v_scale(incident, -1.0), normal);
  FL(5);
  double v = 1.0 - r * r * (1.0 - cos_1 * cos_1);
  *tir = v < 0.0;
  if (*tir) return v_new(0.0, 0.0, 0.0);
  FL(3);   /* sqrt, r * cos_1, - cos_2 */
  double cos_2 = sqrt(v);
  Vec result = v_add(v_scale(incident, r), v_scale(normal, r * cos_1 - cos_2));
  return v_normalized(result);
}

/* Ray-debugger callback (raytracer.rs:17-19; consumer ray_debugger.rs:92-137): when set, each
 * finished ray appends one record, in the reference's callback order. */
typedef struct {
  int depth, ray_type, object, intersected, has_normal, pad;
  double point[3], direction[3], distance, intersection[3], normal[3], color[4];
} OrcRayRecord;
typedef struct { const orc_scene *sc; OrcRayRecord *out; int cap, n; } OrcRec;
static __thread OrcRec *g_rec;

static void debugger_cb(int depth, Ray ray, double distance, const RTObject *obj, Color color, int ray_type) {
  OrcRec *r = g_rec;
  int i = r->n++;
  if (i >= r->cap) return;
  OrcRayRecord *o = &r->out[i];
  memset(o, 0, sizeof *o);
  o->depth = depth; o->ray_type = ray_type; o->distance = distance;
  o->object = obj ? (int)(obj - r->sc->objects) : -1;
  o->intersected = distance != INFINITY;                                           /* ray_debugger.rs:105 */
  Vec ip = v_add(ray.point, v_scale(ray.direction, o->intersected ? distance : 1000.0));
  o->point[0] = ray.point.x; o->point[1] = ray.point.y; o->point[2] = ray.point.z;
  o->direction[0] = ray.direction.x; o->direction[1] = ray.direction.y; o->direction[2] = ray.direction.z;
  o->intersection[0] = ip.x; o->intersection[1] = ip.y; o->intersection[2] = ip.z;
  if (obj) {
    Vec n = shape_get_normal(obj->shape, ip);                                       /* :113-119, not normalised */
    o->has_normal = 1; o->normal[0] = n.x; o->normal[1] = n.y; o->normal[2] = n.z;
  }
  o->color[0] = color.r; o->color[1] = color.g; o->color[2] = color.b; o->color[3] = color.a;
}

static Color get_ray_color(const orc_scene *sc, Ray ray, int depth, int ray_type) { /* raytracer.rs:132-287 */
  NearestCtx nc = {INFINITY, NULL, NULL};
  for (int i = 0; i < sc->n_objects; ++i) {
    nc.cur = &sc->objects[i];
    rtobject_intersects(&sc->objects[i], ray, add_nearest, &nc);
  }
  const RTObject *obj = nc.nearest_obj;
  if (!obj) {                                                                       /* :152-160 */
    if (g_rec) debugger_cb(depth, ray, INFINITY, NULL, BLACK, ray_type);
    return BLACK;
  }
  double nearest_distance = nc.nearest;

  CNT(C_SHADE);
  Vec point = v_add(ray.point, v_scale(ray.direction, nearest_distance));           /* :162 */
  Vec normal = v_normalized(shape_get_normal(obj->shape, point));                  /* :163 */
  UV uv = {0.0, 0.0};
  if (!shape_get_uv(obj->shape, point, &uv)) { uv.u = 0.0; uv.v = 0.0; }            /* :165-168 */
  Color c = mat_color_at(&obj->material, uv);                                       /* :170 */
  Color ambient = c_mul(c, c_intensify(in_range(1.0, 1.0, 1.0), 0.6));              /* :172 */
  Color final_light = ambient;

  for (int li = 0; li < sc->n_lights; ++li) {                                       /* :175-228 */
    const PointLight *light = &sc->lights[li];
    CNT(C_LIGHT); CNT(C_RAY_SHADOW);
    Ray shadow_ray;
    shadow_ray.point = point;
    shadow_ray.direction = v_normalized(v_sub(light->point, point));
    ShadowCtx sh;
    sh.distance = v_length(v_sub(light->point, point));
    sh.transparency = 1.0;
    sh.uv = uv;
    for (int i = 0; i < sc->n_objects; ++i) {
      sh.cached = &sc->objects[i];
      rtobject_intersects(&sc->objects[i], shadow_ray, add_shadow, &sh);
    }
    if (sh.transparency == 0.0) continue;                                           /* :200-202 */
    CNT(C_LIGHT_LIT);
    double angle = v_angle(shadow_ray.direction, normal);
    if (angle >= PI / 2.0) { FL(1); angle = PI - angle; }                           /* :210-214 */
    double intensity = (angle < (PI / 2.0) && angle >= 0.0) ? (FL(2), 1.0 - (angle / (PI / 2.0))) : 0.0;
    Color light_color = c_intensify(c_intensify(light->color, intensity), sh.transparency);
    final_light = c_add(final_light, c_mul(c, light_color));                        /* :227 */
  }

  CNT(C_INSIDE_TEST);
  double angle = v_angle(v_scale(ray.direction, -1.0), normal);                     /* :230 */
  double r1, r2; int inside_out;
  if (angle >= PI / 2.0) { r1 = 1.45; r2 = 1.0; normal = v_scale(normal, -1.0); inside_out = 1; }
  else { r1 = 1.0; r2 = 1.45; inside_out = 0; }

  double transparency = obj->material.transparency;                                 /* :237 */
  double reflectivity = obj->material.reflectivity;                                 /* :238 */
  int tir = 0;

  if (depth < sc->max_depth && transparency != 0.0) {                               /* :242-259 */
    Ray refracted;
    refracted.point = v_add(ray.point, v_scale(ray.direction, nearest_distance));
    FL(1);
    refracted.direction = refracted_dir(ray.direction, normal, r1 / r2, &tir);
    if (!tir) {
      CNT(C_RAY_REFRACT); CNT(C_COMBINE);
      Color rc = get_ray_color(sc, refracted, depth + 1, 2);   /* TransmissionRay */
      FL(1);
      final_light = c_add(c_intensify(final_light, 1.0 - transparency), c_intensify(rc, transparency));
    }
  }
  if (tir) { FL(3); reflectivity = reflectivity + (1.0 - reflectivity) * transparency; } /* :261-265 */

  if (depth < sc->max_depth && reflectivity != 0.0 && (!inside_out || tir)) {       /* :267-280 */
    Ray reflected;
    reflected.point = v_add(ray.point, v_scale(ray.direction, nearest_distance));
    reflected.direction = reflected_dir(ray.direction, normal);
    CNT(C_RAY_REFLECT); CNT(C_COMBINE);
    Color rc = get_ray_color(sc, reflected, depth + 1, 1);   /* ReflectionRay */
    FL(1);
    final_light = c_add(c_intensify(final_light, 1.0 - reflectivity), c_intensify(rc, reflectivity));
  }
  if (g_rec) debugger_cb(depth, ray, nearest_distance, obj, final_light, ray_type);   /* :282-284 */
  return final_light;
}

static Color get_pixel(const orc_scene *sc, double x, double y) {                  /* raytracer.rs:359-363, camera.rs:58-63 */
  CNT(C_RAY_PRIMARY);
  return get_ray_color(sc, camera_create_ray(&sc->camera, x, y), 0, 0);
}

/* ========================================================================= */
/* Scene DSL: scene_grammar.pest + ast_node.rs + context.rs + shape.rs        */
/* ========================================================================= */
typedef enum { V_NONE, V_NUMBER, V_BOOL, V_STRING, V_COLOR, V_VECTOR, V_OBJECT, V_TEXTURE } VKind;
struct ShapeDesc;
typedef struct {
  VKind kind;
  double num;           /* Number; Boolean stored as 0/1 */
  const char *str;
  Color color;          /* Value::Color {r,g,b,a} */
  Vec vec;
  const struct ShapeDesc *shape;
  const Texture *texture;
} Value;

/* sceneparser/shape.rs:7-35 */
typedef enum { SK_SPHERE, SK_CUBE, SK_PLANE, SK_CSG } SKind;
typedef struct ShapeDesc {
  int textured; Color color; const Texture *texture;     /* Material::{Color,Texture} */
  double reflectivity, transparency;
  SKind kind;
  Vec center; double radius;      /* sphere */
  double length;                  /* cube (center shared) */
  Vec normal; double distance;    /* plane */
  CsgOp op; const struct ShapeDesc *a, *b;
  Xform transformation;
} ShapeDesc;

/* ---- AST (ast_node.rs:35-81) ---- */
typedef enum {
  E_VALUE, E_REF, E_VECTOR, E_RGB, E_OBJECT, E_TEXTURE, E_MINUS, E_BINOP
} EKind;
typedef enum { B_ADD, B_SUB, B_MUL, B_DIV, B_MOD, B_LT, B_GT } BinOp;
typedef struct Expr {
  EKind kind;
  Value value;                  /* E_VALUE */
  const char *id;               /* E_REF, E_OBJECT name */
  struct Expr *x, *y, *z;       /* vector/rgb parts; binop a,b in x,y; minus/texture in x */
  BinOp op;
  struct Expr **params; int n_params;   /* E_OBJECT */
} Expr;

typedef enum { S_LIST, S_ASSIGN, S_FUNCTION, S_CALL, S_DRAW, S_XFORM, S_IF, S_WHILE, S_LIGHT, S_CAMERA } SKindStmt;
typedef enum { X_TRANSLATE, X_ROTATE, X_SCALE } XKind;
typedef struct Stmt {
  SKindStmt kind;
  struct Stmt **list; int n_list;        /* S_LIST, function body (as list) */
  int local; const char *id;             /* S_ASSIGN / S_FUNCTION / S_CALL */
  Expr *expr;                            /* assign value, if/while condition, camera position */
  Expr **params; int n_params;           /* call/draw/light */
  const char **param_names; int n_param_names; /* function */
  struct Stmt *body;                     /* function / if / while / transformation statement */
  Expr *x, *y, *z; XKind xkind;
} Stmt;

/* ---- Parser: a PEG restatement of scene_grammar.pest ---- */
typedef struct {
  const char *s; size_t n, pos;
  orc_scene *sc;
  size_t fail_pos;          /* furthest failure, for the error message */
  const char *unimplemented; /* "display"/"append" command seen: ast_node.rs:354 panics in from_pest */
} Parser;

static int p_eof(Parser *p) { return p->pos >= p->n; }
static char p_peek(Parser *p, size_t off) { return p->pos + off < p->n ? p->s[p->pos + off] : '\0'; }
static void p_fail(Parser *p) { if (p->pos > p->fail_pos) p->fail_pos = p->pos; }
static int is_alpha_c(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }
static int is_digit_c(char c) { return c >= '0' && c <= '9'; }
static int is_alnum_c(char c) { return is_alpha_c(c) || is_digit_c(c) || c == '_'; }  /* pest:8 */

/* WHITESPACE = _{ " " | "\n" | "\r" | comment }   (pest:2-3) -- one token */
static int p_ws1(Parser *p) {
  char c = p_peek(p, 0);
  if (c == ' ' || c == '\n' || c == '\r') { p->pos++; return 1; }
  if (c == '/' && p_peek(p, 1) == '/') {
    p->pos += 2;
    while (!p_eof(p) && p->s[p->pos] != '\n') p->pos++;
    if (!p_eof(p)) p->pos++;  /* "\n" (the (!"\n" ANY)* loop also ate any "\r") */
    return 1;
  }
  return 0;
}
static void p_ws(Parser *p) { while (p_ws1(p)) {} }

static int p_lit(Parser *p, const char *lit) {           /* literal string, no whitespace */
  size_t l = strlen(lit);
  if (p->pos + l <= p->n && memcmp(p->s + p->pos, lit, l) == 0) { p->pos += l; return 1; }
  p_fail(p);
  return 0;
}
/* keyword ~ !alnum */
static int p_kw(Parser *p, const char *kw) {
  size_t save = p->pos;
  if (!p_lit(p, kw)) return 0;
  if (is_alnum_c(p_peek(p, 0))) { p->pos = save; p_fail(p); return 0; }
  return 1;
}
static int p_kw_any(Parser *p, const char *const *kws, int n, const char **which) {
  for (int i = 0; i < n; ++i) if (p_kw(p, kws[i])) { if (which) *which = kws[i]; return 1; }
  return 0;
}
static const char *const K_COMMAND[] = {"draw", "display", "append"};              /* pest:44 */
static const char *const K_OBJ[] = {"sphere", "plane", "csg", "cube"};             /* pest:45 */
static const char *const K_XFORM[] = {"scale", "rotate", "translate"};             /* pest:46 */
static const char *const K_COLOR[] = {"red", "orange", "yellow", "green", "blue", "purple", "black", "white"}; /* pest:47 */

/* keyword = @{ local_ | transformation_ | command_ | obj_name | function_ } (pest:50) */
static int p_keyword_ahead(Parser *p) {
  size_t save = p->pos;
  int r = p_kw(p, "local") || p_kw_any(p, K_XFORM, 3, NULL) || p_kw_any(p, K_COMMAND, 3, NULL) ||
          p_kw_any(p, K_OBJ, 4, NULL) || p_kw(p, "function");
  p->pos = save;
  return r;
}
/* id = @{ !keyword ~ ident }; ident = @{ (alpha | "_") ~ alnum* }  (pest:9, 51-52) */
static const char *p_id(Parser *p) {
  if (p_keyword_ahead(p)) { p_fail(p); return NULL; }
  char c = p_peek(p, 0);
  if (!(is_alpha_c(c) || c == '_')) { p_fail(p); return NULL; }
  size_t st = p->pos;
  while (is_alnum_c(p_peek(p, 0))) p->pos++;
  char *r = (char *)arena_alloc(p->sc, p->pos - st + 1);
  memcpy(r, p->s + st, p->pos - st);
  return r;
}

static Expr *new_expr(Parser *p, EKind k) { Expr *e = (Expr *)arena_alloc(p->sc, sizeof(Expr)); e->kind = k; return e; }
static Stmt *new_stmt(Parser *p, SKindStmt k) { Stmt *s = (Stmt *)arena_alloc(p->sc, sizeof(Stmt)); s->kind = k; return s; }

typedef struct { void **v; int n, cap; } PtrVec;
static void pv_push(PtrVec *pv, void *x) {
  if (pv->n == pv->cap) { pv->cap = pv->cap ? 2 * pv->cap : 8; pv->v = (void **)realloc(pv->v, sizeof(void *) * pv->cap); }
  pv->v[pv->n++] = x;
}
static void **pv_freeze(Parser *p, PtrVec *pv) {
  void **r = (void **)arena_alloc(p->sc, sizeof(void *) * (pv->n ? pv->n : 1));
  if (pv->n) memcpy(r, pv->v, sizeof(void *) * pv->n);
  free(pv->v);
  return r;
}

static Expr *p_expression(Parser *p);
static Stmt *p_statement(Parser *p);
static Stmt *p_statement_list(Parser *p);

/* param_list = { (expression ~ ","?)* }  (pest:30) */
static Expr **p_param_list(Parser *p, int *n) {
  PtrVec pv = {0};
  for (;;) {
    size_t save = p->pos;
    if (pv.n) p_ws(p);
    Expr *e = p_expression(p);
    if (!e) { p->pos = save; break; }
    pv_push(&pv, e);
    size_t s2 = p->pos;
    p_ws(p);
    if (!p_lit(p, ",")) p->pos = s2;
  }
  *n = pv.n;
  return (Expr **)pv_freeze(p, &pv);
}
/* number_literal = @{ digit+ ~ ("." ~ digit+)? ~ !alpha }  (pest:53) */
static Expr *p_number(Parser *p) {
  size_t st = p->pos;
  if (!is_digit_c(p_peek(p, 0))) { p_fail(p); return NULL; }
  while (is_digit_c(p_peek(p, 0))) p->pos++;
  if (p_peek(p, 0) == '.' && is_digit_c(p_peek(p, 1))) {
    p->pos++;
    while (is_digit_c(p_peek(p, 0))) p->pos++;
  }
  if (is_alpha_c(p_peek(p, 0))) { p->pos = st; p_fail(p); return NULL; }
  char buf[512];
  size_t l = p->pos - st;
  if (l >= sizeof buf) l = sizeof buf - 1;
  memcpy(buf, p->s + st, l); buf[l] = 0;
  Expr *e = new_expr(p, E_VALUE);
  e->value.kind = V_NUMBER;
  e->value.num = strtod(buf, NULL);   /* str::parse::<f64> (ast_node.rs:658-660): correctly rounded */
  return e;
}
/* string_literal (pest:54) */
static Expr *p_string(Parser *p) {
  char q = p_peek(p, 0);
  if (q != '"' && q != '\'') { p_fail(p); return NULL; }
  size_t st = p->pos + 1, e = st;
  while (e < p->n && p->s[e] != q) e++;
  if (e >= p->n) { p_fail(p); return NULL; }
  char *str = (char *)arena_alloc(p->sc, e - st + 1);
  memcpy(str, p->s + st, e - st);
  p->pos = e + 1;
  Expr *x = new_expr(p, E_VALUE);
  x->value.kind = V_STRING; x->value.str = str;
  return x;
}
/* value = { number_literal | color_name | color | vector | texture | ("(" ~ expression ~ ")")
 *           | object | string_literal | id_reference }   (pest:71-74) */
static Expr *p_value(Parser *p) {
  size_t save = p->pos;
  Expr *e;
  const char *which;
  if ((e = p_number(p))) return e;
  p->pos = save;
  if (p_kw_any(p, K_COLOR, 8, &which)) {                                            /* ast_node.rs:661-675 */
    static const double cols[8][3] = {{1, 0, 0}, {1, 0.5, 0}, {1, 1, 0}, {0, 1, 0}, {0, 0, 1}, {1, 0, 1}, {0, 0, 0}, {1, 1, 1}};
    int k = 0;
    while (strcmp(K_COLOR[k], which)) k++;
    e = new_expr(p, E_VALUE);
    e->value.kind = V_COLOR;
    e->value.color.r = cols[k][0]; e->value.color.g = cols[k][1]; e->value.color.b = cols[k][2]; e->value.color.a = 1.0;
    return e;
  }
  p->pos = save;
  /* color = { "rgb" ~ "(" ~ (expression ~ ","?){3} ~ ")" } (pest:57) */
  if (p_lit(p, "rgb")) {
    p_ws(p);
    if (p_lit(p, "(")) {
      Expr *parts[3]; int ok = 1;
      for (int i = 0; i < 3 && ok; ++i) {
        p_ws(p);
        parts[i] = p_expression(p);
        if (!parts[i]) { ok = 0; break; }
        size_t s2 = p->pos; p_ws(p); if (!p_lit(p, ",")) p->pos = s2;
      }
      if (ok) { p_ws(p); if (p_lit(p, ")")) { e = new_expr(p, E_RGB); e->x = parts[0]; e->y = parts[1]; e->z = parts[2]; return e; } }
    }
  }
  p->pos = save;
  /* vector = { "<" ~ expression ~ "," ~ expression ~ "," ~ expression ~ ">" } (pest:58) */
  if (p_lit(p, "<")) {
    Expr *x, *y, *z;
    p_ws(p);
    if ((x = p_expression(p))) { p_ws(p); if (p_lit(p, ",")) { p_ws(p);
      if ((y = p_expression(p))) { p_ws(p); if (p_lit(p, ",")) { p_ws(p);
        if ((z = p_expression(p))) { p_ws(p); if (p_lit(p, ">")) {
          e = new_expr(p, E_VECTOR); e->x = x; e->y = y; e->z = z; return e; } } } } } }
  }
  p->pos = save;
  /* texture = { "texture" ~ "(" ~ expression ~ ")" } (pest:60) */
  if (p_lit(p, "texture")) {
    p_ws(p);
    if (p_lit(p, "(")) { p_ws(p); Expr *x = p_expression(p);
      if (x) { p_ws(p); if (p_lit(p, ")")) { e = new_expr(p, E_TEXTURE); e->x = x; return e; } } }
  }
  p->pos = save;
  if (p_lit(p, "(")) {
    p_ws(p);
    Expr *x = p_expression(p);
    if (x) { p_ws(p); if (p_lit(p, ")")) return x; }
  }
  p->pos = save;
  /* object = { obj_name ~ "(" ~ param_list ~ ")" } (pest:59) */
  if (p_kw_any(p, K_OBJ, 4, &which)) {
    p_ws(p);
    if (p_lit(p, "(")) {
      int n; p_ws(p);
      Expr **params = p_param_list(p, &n);
      p_ws(p);
      if (p_lit(p, ")")) { e = new_expr(p, E_OBJECT); e->id = which; e->params = params; e->n_params = n; return e; }
    }
  }
  p->pos = save;
  if ((e = p_string(p))) return e;
  p->pos = save;
  const char *id = p_id(p);                                                         /* id_reference */
  if (id) { e = new_expr(p, E_REF); e->id = id; return e; }
  p->pos = save;
  return NULL;
}
/* neg_expression = { minus? ~ value } (pest:69) */
static Expr *p_neg(Parser *p) {
  size_t save = p->pos;
  int minus = 0;
  if (p_peek(p, 0) == '-') { p->pos++; minus = 1; p_ws(p); }
  Expr *v = p_value(p);
  if (!v) { p->pos = save; return NULL; }
  if (!minus) return v;
  Expr *e = new_expr(p, E_MINUS); e->x = v;
  return e;
}
/* mult_expression / expression: only the FIRST operator and right operand are kept; the rest of an
 * `a op b op c` chain is parsed and silently dropped (ast_node.rs:598-629). */
static Expr *p_chain(Parser *p, Expr *(*sub)(Parser *), const char *ops) {
  Expr *left = sub(p);
  if (!left) return NULL;
  Expr *result = left;
  int first = 1;
  for (;;) {
    size_t save = p->pos;
    p_ws(p);
    char c = p_peek(p, 0);
    if (!c || !strchr(ops, c)) { p->pos = save; break; }
    p->pos++;
    p_ws(p);
    Expr *right = sub(p);
    if (!right) { p->pos = save; break; }
    if (first) {
      Expr *e = new_expr(p, E_BINOP);
      e->op = c == '+' ? B_ADD : c == '-' ? B_SUB : c == '*' ? B_MUL : c == '/' ? B_DIV : B_MOD;
      e->x = left; e->y = right;
      result = e; first = 0;
    }
  }
  return result;
}
static Expr *p_mult(Parser *p) { return p_chain(p, p_neg, "*/%"); }                /* pest:68 */
static Expr *p_expression(Parser *p) { return p_chain(p, p_mult, "+-"); }          /* pest:67 */
/* bool_expression = { expression ~ bool_operator ~ expression } (pest:66) */
static Expr *p_bool_expression(Parser *p) {
  size_t save = p->pos;
  Expr *a = p_expression(p);
  if (!a) return NULL;
  p_ws(p);
  char c = p_peek(p, 0);
  if (c != '<' && c != '>') { p_fail(p); p->pos = save; return NULL; }
  p->pos++;
  p_ws(p);
  Expr *b = p_expression(p);
  if (!b) { p->pos = save; return NULL; }
  Expr *e = new_expr(p, E_BINOP);
  e->op = c == '<' ? B_LT : B_GT; e->x = a; e->y = b;
  return e;
}

/* Statements (pest:17-27) */
static Stmt *p_statement(Parser *p) {
  size_t save = p->pos;
  /* set_camera_statement = { set_camera_ ~ "(" ~ expression ~ ")" }, set_camera_ = @{"set" ~ WHITESPACE ~ "camera" ~ !alnum} */
  if (p_lit(p, "set") && p_ws1(p) && p_kw(p, "camera")) {
    p_ws(p);
    if (p_lit(p, "(")) { p_ws(p); Expr *e = p_expression(p);
      if (e) { p_ws(p); if (p_lit(p, ")")) { Stmt *s = new_stmt(p, S_CAMERA); s->expr = e; return s; } } }
  }
  p->pos = save;
  /* append_light_statement = { append_light_ ~ "(" ~ param_list ~ ")" } */
  if (p_lit(p, "append") && p_ws1(p) && p_kw(p, "light")) {
    p_ws(p);
    if (p_lit(p, "(")) { int n; p_ws(p); Expr **pl = p_param_list(p, &n); p_ws(p);
      if (p_lit(p, ")")) { Stmt *s = new_stmt(p, S_LIGHT); s->params = pl; s->n_params = n; return s; } }
  }
  p->pos = save;
  /* do_statement = { do_ ~ statement_list ~ end_ } */
  if (p_kw(p, "do")) {
    p_ws(p);
    Stmt *l = p_statement_list(p);
    p_ws(p);
    if (p_kw(p, "end")) return l;
  }
  p->pos = save;
  /* if_statement / while_statement */
  for (int w = 0; w < 2; ++w) {
    if (p_kw(p, w ? "while" : "if")) {
      p_ws(p);
      Expr *c = p_bool_expression(p);
      if (c) { p_ws(p);
        if (p_kw(p, w ? "do" : "then")) { p_ws(p);
          Stmt *l = p_statement_list(p); p_ws(p);
          if (p_kw(p, "end")) { Stmt *s = new_stmt(p, w ? S_WHILE : S_IF); s->expr = c; s->body = l; return s; } } }
    }
    p->pos = save;
  }
  /* call_statement = { call_ ~ id ~ "(" ~ param_list ~ ")" } */
  if (p_kw(p, "call")) {
    p_ws(p);
    const char *id = p_id(p);
    if (id) { p_ws(p); if (p_lit(p, "(")) { int n; p_ws(p); Expr **pl = p_param_list(p, &n); p_ws(p);
      if (p_lit(p, ")")) { Stmt *s = new_stmt(p, S_CALL); s->id = id; s->params = pl; s->n_params = n; return s; } } }
  }
  p->pos = save;
  /* function_statement = { function_ ~ id ~ "(" ~ (id ~ ","?)* ~ ")" ~ statement_list ~ end_ } */
  if (p_kw(p, "function")) {
    p_ws(p);
    const char *id = p_id(p);
    if (id) { p_ws(p); if (p_lit(p, "(")) {
      PtrVec names = {0};
      for (;;) {
        size_t s2 = p->pos;
        p_ws(p);
        const char *pn = p_id(p);
        if (!pn) { p->pos = s2; break; }
        pv_push(&names, (void *)pn);
        size_t s3 = p->pos; p_ws(p); if (!p_lit(p, ",")) p->pos = s3;
      }
      int nn = names.n;
      const char **pnames = (const char **)pv_freeze(p, &names);
      p_ws(p);
      if (p_lit(p, ")")) { p_ws(p); Stmt *l = p_statement_list(p); p_ws(p);
        if (p_kw(p, "end")) { Stmt *s = new_stmt(p, S_FUNCTION); s->id = id; s->param_names = pnames; s->n_param_names = nn; s->body = l; return s; } } } }
  }
  p->pos = save;
  /* command_statement = { command_ ~ "(" ~ param_list ~ ")" } */
  {
    const char *which;
    if (p_kw_any(p, K_COMMAND, 3, &which)) {
      p_ws(p);
      if (p_lit(p, "(")) { int n; p_ws(p); Expr **pl = p_param_list(p, &n); p_ws(p);
        if (p_lit(p, ")")) {
          Stmt *s = new_stmt(p, S_DRAW); s->id = which; s->params = pl; s->n_params = n;
          if (strcmp(which, "draw")) p->unimplemented = which;
          return s; } }
    }
  }
  p->pos = save;
  /* assignment_statement = { local_? ~ id ~ "=" ~ expression } */
  {
    int local = 0;
    if (p_kw(p, "local")) { local = 1; p_ws(p); }
    const char *id = p_id(p);
    if (id) { p_ws(p); if (p_lit(p, "=")) { p_ws(p); Expr *e = p_expression(p);
      if (e) { Stmt *s = new_stmt(p, S_ASSIGN); s->local = local; s->id = id; s->expr = e; return s; } } }
  }
  p->pos = save;
  /* transformation_statement = { transformation_ ~ "(" ~ e ~ "," ~ e ~ "," ~ e ~ ")" ~ statement } */
  {
    const char *which;
    if (p_kw_any(p, K_XFORM, 3, &which)) {
      p_ws(p);
      Expr *x, *y, *z;
      if (p_lit(p, "(")) { p_ws(p); if ((x = p_expression(p))) { p_ws(p); if (p_lit(p, ",")) { p_ws(p);
        if ((y = p_expression(p))) { p_ws(p); if (p_lit(p, ",")) { p_ws(p);
          if ((z = p_expression(p))) { p_ws(p); if (p_lit(p, ")")) { p_ws(p);
            Stmt *body = p_statement(p);
            if (body) {
              Stmt *s = new_stmt(p, S_XFORM);
              s->x = x; s->y = y; s->z = z; s->body = body;
              s->xkind = which[0] == 't' ? X_TRANSLATE : which[0] == 'r' ? X_ROTATE : X_SCALE;
              return s; } } } } } } } }
    }
  }
  p->pos = save;
  return NULL;
}
/* statement_list = { statement* } */
static Stmt *p_statement_list(Parser *p) {
  PtrVec pv = {0};
  for (;;) {
    size_t save = p->pos;
    if (pv.n) p_ws(p);
    Stmt *s = p_statement(p);
    if (!s) { p->pos = save; break; }
    pv_push(&pv, s);
  }
  Stmt *l = new_stmt(p, S_LIST);
  l->n_list = pv.n;
  l->list = (Stmt **)pv_freeze(p, &pv);
  return l;
}

/* ---- Evaluator (ast_node.rs:150-265, 438-596; context.rs) ---- */
typedef struct VarEntry { const char *name; Value value; struct VarEntry *next; } VarEntry;
typedef struct { VarEntry *head; } VarMap;
typedef struct FuncEntry { const char *name; const Stmt *def; struct FuncEntry *next; } FuncEntry;

typedef struct {
  orc_scene *sc;
  VarMap globals;
  VarMap *stack; int n_stack, cap_stack;
  FuncEntry *functions;
  char err[512];
  int failed;
} Ctx;

static Value *map_get(VarMap *m, const char *name) {
  for (VarEntry *e = m->head; e; e = e->next) if (!strcmp(e->name, name)) return &e->value;
  return NULL;
}
static void map_insert(Ctx *c, VarMap *m, const char *name, Value v) {
  Value *old = map_get(m, name);
  if (old) { *old = v; return; }
  VarEntry *e = (VarEntry *)arena_alloc(c->sc, sizeof(VarEntry));
  e->name = name; e->value = v; e->next = m->head; m->head = e;
}
static VarMap *ctx_locals(Ctx *c) { return c->n_stack ? &c->stack[c->n_stack - 1] : &c->globals; } /* context.rs:26-32 */

static void fail(Ctx *c, const char *fmt, ...) {
  if (c->failed) return;
  c->failed = 1;
  va_list ap; va_start(ap, fmt);
  vsnprintf(c->err, sizeof c->err, fmt, ap);
  va_end(ap);
}
static const Xform *cur_xform(Ctx *c) { return &c->sc->xstack[c->sc->n_x - 1]; }
static void push_xform(Ctx *c, Xform t) {                                           /* transformation.rs:21-28 */
  orc_scene *sc = c->sc;
  Xform n = xf_compose_with(&t, &sc->xstack[sc->n_x - 1]);
  if (sc->n_x == sc->cap_x) { sc->cap_x *= 2; sc->xstack = (Xform *)realloc(sc->xstack, sizeof(Xform) * sc->cap_x); }
  sc->xstack[sc->n_x++] = n;
}
static void pop_xform(Ctx *c) { c->sc->n_x--; }

static double to_number(Ctx *c, Value v) {                                          /* value.rs:16-22 */
  if (v.kind != V_NUMBER) { fail(c, "Cannot convert value to number"); return 0.0; }
  return v.num;
}

static Value eval(Ctx *c, const Expr *e);

typedef struct {              /* ValuesByType (ast_node.rs:105-148) */
  double num[64]; int n_num, i_num;
  const char *str[16]; int n_str, i_str;
  Vec vec[16]; int n_vec, i_vec;
  const ShapeDesc *obj[16]; int n_obj, i_obj;
  Color col[16]; int n_col, i_col;
  const Texture *tex[16]; int n_tex, i_tex;
} Bucket;
static void bucket_fill(Ctx *c, Bucket *b, Expr **params, int n) {
  memset(b, 0, sizeof *b);
  for (int i = 0; i < n && !c->failed; ++i) {
    Value v = eval(c, params[i]);
    switch (v.kind) {
      case V_NUMBER: if (b->n_num < 64) b->num[b->n_num++] = v.num; break;
      case V_STRING: if (b->n_str < 16) b->str[b->n_str++] = v.str; break;
      case V_COLOR: if (b->n_col < 16) b->col[b->n_col++] = v.color; break;
      case V_VECTOR: if (b->n_vec < 16) b->vec[b->n_vec++] = v.vec; break;
      case V_OBJECT: if (b->n_obj < 16) b->obj[b->n_obj++] = v.shape; break;
      case V_TEXTURE: if (b->n_tex < 16) b->tex[b->n_tex++] = v.texture; break;
      default: fail(c, "Unexpected argument type: boolean");
    }
  }
}

static Value eval(Ctx *c, const Expr *e) {
  Value r; memset(&r, 0, sizeof r);
  if (c->failed) return r;
  switch (e->kind) {
    case E_VALUE: return e->value;
    case E_REF: {                                                                   /* ast_node.rs:442-451 */
      Value *v = map_get(ctx_locals(c), e->id);
      if (!v) v = map_get(&c->globals, e->id);
      if (!v) { fail(c, "Didn't find variable %s", e->id); return r; }
      return *v;
    }
    case E_VECTOR: {                                                                /* :452-458 */
      double x = to_number(c, eval(c, e->x)), y = to_number(c, eval(c, e->y)), z = to_number(c, eval(c, e->z));
      r.kind = V_VECTOR; r.vec = v_new(x, y, z);
      return r;
    }
    case E_RGB: {                                                                   /* :459-465 */
      double x = to_number(c, eval(c, e->x)), y = to_number(c, eval(c, e->y)), z = to_number(c, eval(c, e->z));
      r.kind = V_COLOR; r.color.r = x; r.color.g = y; r.color.b = z; r.color.a = 1.0;
      return r;
    }
    case E_OBJECT: {                                                                /* :466-528 */
      Bucket b;
      bucket_fill(c, &b, e->params, e->n_params);
      if (c->failed) return r;
      ShapeDesc *s = (ShapeDesc *)arena_alloc(c->sc, sizeof(ShapeDesc));
      const char *name = e->id;
      if (!strcmp(name, "sphere")) {
        s->kind = SK_SPHERE;
        s->center = b.i_vec < b.n_vec ? b.vec[b.i_vec++] : v_new(0, 0, 0);
        s->radius = b.i_num < b.n_num ? b.num[b.i_num++] : 1.0;
      } else if (!strcmp(name, "cube")) {
        s->kind = SK_CUBE;
        s->center = b.i_vec < b.n_vec ? b.vec[b.i_vec++] : v_new(0, 0, 0);
        s->length = b.i_num < b.n_num ? b.num[b.i_num++] : 1.0;
      } else if (!strcmp(name, "plane")) {
        s->kind = SK_PLANE;
        s->normal = b.i_vec < b.n_vec ? b.vec[b.i_vec++] : v_new(0, 1, 0);
        s->distance = b.i_num < b.n_num ? b.num[b.i_num++] : 1.0;
      } else {
        s->kind = SK_CSG;
        const char *op = b.i_str < b.n_str ? b.str[b.i_str++] : "union";
        if (!strcmp(op, "union")) s->op = OP_UNION;
        else if (!strcmp(op, "intersection")) s->op = OP_INTERSECTION;
        else if (!strcmp(op, "difference")) s->op = OP_DIFFERENCE;
        else { fail(c, "Unknown CSG operator: %s", op); return r; }
        if (b.i_obj >= b.n_obj) { fail(c, "Expected object 1!"); return r; }
        s->a = b.obj[b.i_obj++];
        if (b.i_obj >= b.n_obj) { fail(c, "Expected object 2!"); return r; }
        s->b = b.obj[b.i_obj++];
      }
      s->transformation = *cur_xform(c);
      if (b.i_tex < b.n_tex) { s->textured = 1; s->texture = b.tex[b.i_tex++]; }
      else { s->textured = 0; s->color = b.i_col < b.n_col ? b.col[b.i_col++] : BLACK; }
      s->reflectivity = b.i_num < b.n_num ? b.num[b.i_num++] : 0.0;
      s->transparency = b.i_num < b.n_num ? b.num[b.i_num++] : 0.0;
      if (b.i_num != b.n_num || b.i_str != b.n_str || b.i_vec != b.n_vec || b.i_obj != b.n_obj ||
          b.i_col != b.n_col || b.i_tex != b.n_tex) {                               /* assert_empty (:139-147) */
        fail(c, "assertion failed: unused object arguments");
        return r;
      }
      r.kind = V_OBJECT; r.shape = s;
      return r;
    }
    case E_TEXTURE: {                                                               /* :529-532 */
      Value f = eval(c, e->x);
      if (f.kind != V_STRING) { fail(c, "Cannot convert value to string"); return r; }
      const Texture *t = find_texture(f.str);
      if (!t) { fail(c, "texture '%s' not registered with the oracle", f.str); return r; }
      r.kind = V_TEXTURE; r.texture = t;
      return r;
    }
    case E_MINUS: {                                                                 /* :533-542 */
      Value v = eval(c, e->x);
      if (v.kind == V_NUMBER) { v.num = -v.num; return v; }
      if (v.kind == V_VECTOR) { v.vec = v_new(-v.vec.x, -v.vec.y, -v.vec.z); return v; }
      fail(c, "Cannot apply - to value");
      return r;
    }
    case E_BINOP: {                                                                 /* :543-594 */
      Value a = eval(c, e->x), b = eval(c, e->y);
      if (c->failed) return r;
      switch (e->op) {
        case B_ADD: r.kind = V_NUMBER; r.num = to_number(c, a) + to_number(c, b); return r;
        case B_SUB: r.kind = V_NUMBER; r.num = to_number(c, a) - to_number(c, b); return r;
        case B_MUL: case B_DIV: {
          int div = e->op == B_DIV;
          if (a.kind == V_NUMBER && b.kind == V_NUMBER) { r.kind = V_NUMBER; r.num = div ? a.num / b.num : a.num * b.num; return r; }
          const Value *cv = a.kind == V_COLOR ? &a : b.kind == V_COLOR ? &b : NULL;
          const Value *vv = a.kind == V_VECTOR ? &a : b.kind == V_VECTOR ? &b : NULL;
          const Value *nv = a.kind == V_NUMBER ? &a : b.kind == V_NUMBER ? &b : NULL;
          if (cv && nv) {
            double x = nv->num; Color k = cv->color;
            r.kind = V_COLOR;
            if (div) { r.color.r = k.r / x; r.color.g = k.g / x; r.color.b = k.b / x; r.color.a = k.a / x; }
            else { r.color.r = k.r * x; r.color.g = k.g * x; r.color.b = k.b * x; r.color.a = k.a * x; }
            return r;
          }
          if (vv && nv) {
            double x = nv->num; Vec k = vv->vec;
            r.kind = V_VECTOR;
            r.vec = div ? v_new(k.x / x, k.y / x, k.z / x) : v_new(k.x * x, k.y * x, k.z * x);
            return r;
          }
          fail(c, div ? "Cannot divide values" : "Cannot multiply values");
          return r;
        }
        case B_GT: case B_LT:
          if (a.kind != V_NUMBER || b.kind != V_NUMBER) { fail(c, "Cannot compare values"); return r; }
          r.kind = V_BOOL; r.num = e->op == B_GT ? (a.num > b.num) : (a.num < b.num);
          return r;
        default: fail(c, "Operator Modulo not yet implemented"); return r;
      }
    }
  }
  return r;
}

/* Shape::to_rt_object (sceneparser/shape.rs:42-93) */
static RTObject *to_rt_object(Ctx *c, const ShapeDesc *d) {
  RTObject *o = (RTObject *)arena_alloc(c->sc, sizeof(RTObject));
  o->material.textured = d->textured;
  o->material.color = d->color;
  o->material.texture = d->texture;
  o->material.reflectivity = d->reflectivity;
  o->material.transparency = d->transparency;
  Shape *s = (Shape *)arena_alloc(c->sc, sizeof(Shape));
  s->t = d->transformation;
  switch (d->kind) {
    case SK_SPHERE: s->kind = SH_SPHERE; s->center = d->center; s->radius = d->radius; break;
    case SK_CUBE: s->kind = SH_CUBE; cube_init(s, d->transformation, d->center, d->length); break;
    case SK_PLANE:                                                                  /* MathPlane::from_normal */
      s->kind = SH_PLANE;
      s->plane = plane_new(d->transformation, d->normal.x, d->normal.y, d->normal.z, d->distance);
      break;
    case SK_CSG:
      s->kind = SH_CSG; s->op = d->op;
      s->a_obj = to_rt_object(c, d->a);
      s->b_obj = to_rt_object(c, d->b);
      break;
  }
  o->shape = s;
  return o;
}

static void exec(Ctx *c, const Stmt *s) {
  if (c->failed) return;
  orc_scene *sc = c->sc;
  switch (s->kind) {
    case S_LIST:
      for (int i = 0; i < s->n_list && !c->failed; ++i) exec(c, s->list[i]);
      break;
    case S_ASSIGN: {                                                                /* ast_node.rs:158-165 */
      Value v = eval(c, s->expr);
      if (c->failed) return;
      map_insert(c, s->local ? ctx_locals(c) : &c->globals, s->id, v);
      break;
    }
    case S_FUNCTION: {                                                              /* :166-168 */
      FuncEntry *f;
      for (f = c->functions; f; f = f->next) if (!strcmp(f->name, s->id)) break;
      if (!f) { f = (FuncEntry *)arena_alloc(sc, sizeof(FuncEntry)); f->name = s->id; f->next = c->functions; c->functions = f; }
      f->def = s;
      break;
    }
    case S_CALL: {                                                                  /* :169-175, context.rs:49-62 */
      Value vals[64];
      int n = s->n_params < 64 ? s->n_params : 64;
      for (int i = 0; i < n; ++i) vals[i] = eval(c, s->params[i]);
      if (c->failed) return;
      FuncEntry *f;
      for (f = c->functions; f; f = f->next) if (!strcmp(f->name, s->id)) break;
      if (!f) { fail(c, "called `Option::unwrap()` on a `None` value (function %s)", s->id); return; }
      if (f->def->n_param_names != n) { fail(c, "assertion failed: param count for %s", s->id); return; }
      if (c->n_stack == c->cap_stack) {
        c->cap_stack = c->cap_stack ? 2 * c->cap_stack : 16;
        c->stack = (VarMap *)realloc(c->stack, sizeof(VarMap) * c->cap_stack);
      }
      c->stack[c->n_stack++].head = NULL;
      for (int i = 0; i < n; ++i) map_insert(c, ctx_locals(c), f->def->param_names[i], vals[i]);
      exec(c, f->def->body);
      c->n_stack--;
      break;
    }
    case S_DRAW: {                                                                  /* :176-191, 343-357 */
      if (strcmp(s->id, "draw")) { fail(c, "not implemented: %s", s->id); return; }
      Value vals[64];
      int n = s->n_params < 64 ? s->n_params : 64;
      for (int i = 0; i < n; ++i) vals[i] = eval(c, s->params[i]);
      if (c->failed) return;
      if (s->n_params != 1) { fail(c, "assertion failed: draw takes one value"); return; }
      if (vals[0].kind != V_OBJECT) { fail(c, "Didn't get an object on draw!"); return; }
      RTObject *o = to_rt_object(c, vals[0].shape);
      if (sc->n_objects == sc->cap_objects) {
        sc->cap_objects = sc->cap_objects ? 2 * sc->cap_objects : 16;
        sc->objects = (RTObject *)realloc(sc->objects, sizeof(RTObject) * sc->cap_objects);
      }
      sc->objects[sc->n_objects++] = *o;                                            /* raytracer.rs:309-311 */
      break;
    }
    case S_XFORM: {                                                                 /* :192-219 */
      double x = to_number(c, eval(c, s->x));
      double y = to_number(c, eval(c, s->y));
      double z = to_number(c, eval(c, s->z));
      if (c->failed) return;
      Xform t = s->xkind == X_TRANSLATE ? xf_translation(x, y, z)
              : s->xkind == X_ROTATE ? xf_rotation(x, y, z) : xf_scaling(x, y, z);
      push_xform(c, t);
      exec(c, s->body);
      pop_xform(c);
      break;
    }
    case S_IF: case S_WHILE: {                                                      /* :220-229 */
      for (;;) {
        Value v = eval(c, s->expr);
        if (c->failed) return;
        if (v.kind != V_BOOL) { fail(c, "Cannot convert value to boolean"); return; }
        if (!v.num) break;
        exec(c, s->body);
        if (c->failed || s->kind == S_IF) break;
      }
      break;
    }
    case S_LIGHT: {                                                                 /* :230-251 */
      Bucket b;
      bucket_fill(c, &b, s->params, s->n_params);
      if (c->failed) return;
      PointLight L;
      if (b.n_col) L.color = b.col[0]; else { L.color.r = 0.5; L.color.g = 0.5; L.color.b = 0.5; L.color.a = 1.0; }
      Vec pt = b.n_vec ? b.vec[0] : v_new(0, 0, 0);
      L.fade_distance = b.n_num ? b.num[0] : 100.0;
      L.point = xf_transform_vector(cur_xform(c), pt);
      if (sc->n_lights == sc->cap_lights) {
        sc->cap_lights = sc->cap_lights ? 2 * sc->cap_lights : 8;
        sc->lights = (PointLight *)realloc(sc->lights, sizeof(PointLight) * sc->cap_lights);
      }
      sc->lights[sc->n_lights++] = L;
      break;
    }
    case S_CAMERA: {                                                                /* :252-263 */
      Value v = eval(c, s->expr);
      if (c->failed) return;
      if (v.kind != V_VECTOR) { fail(c, "Cannot convert value to vector"); return; }
      Vec pos = xf_transform_vector(cur_xform(c), v.vec);
      Vec center = xf_transform_vector(cur_xform(c), pos);                         /* raytracer.rs:289-299 */
      sc->camera = camera_new(sc->width, sc->height, center);
      break;
    }
  }
}

/* ========================================================================= */
/* Public API                                                                 */
/* ========================================================================= */
static void scene_defaults(orc_scene *sc, int width, int height) {
  /* RayTracer::new_default (raytracer.rs:38-70) + add_test_objects (:125-129) */
  sc->width = width; sc->height = height; sc->max_depth = 10;
  sc->camera = camera_new(width, height, v_new(0.0, 0.0, -100.0));
  sc->cap_x = 16; sc->n_x = 1;
  sc->xstack = (Xform *)malloc(sizeof(Xform) * sc->cap_x);
  sc->xstack[0] = xf_identity();
  PointLight L;
  L.point = v_new(-10.0, 30.0, -50.0);
  L.color = in_range(0.5, 0.5, 0.5);
  L.fade_distance = 100.0;
  sc->cap_lights = 8; sc->n_lights = 1;
  sc->lights = (PointLight *)malloc(sizeof(PointLight) * sc->cap_lights);
  sc->lights[0] = L;
}

void orc_free_scene(orc_scene *sc) {
  if (!sc) return;
  free(sc->objects); free(sc->lights); free(sc->xstack);
  Arena *a = sc->arena;
  while (a) { Arena *n = a->next; free(a); a = n; }
  free(sc);
}

/* load_scene (scene_loader.rs:24-47) on a fresh RayTracer (debug_window.rs:53-62).
 * Returns NULL with err set on a runtime error (the reference panics).  On a *parse*
 * error the reference prints the error and renders the default scene: status 1 and a
 * default scene are returned. */
orc_scene *orc_load_scene(const char *text, double time, int width, int height, int *status,
                          char *err, int errlen) {
  orc_scene *sc = (orc_scene *)calloc(1, sizeof *sc);
  scene_defaults(sc, width, height);
  if (status) *status = 0;
  if (err && errlen) err[0] = 0;
  Parser p = {text, strlen(text), 0, sc, 0, NULL};
  /* scene = _{ SOI ~ statement_list ~ EOI } */
  p_ws(&p);
  Stmt *ast = p_statement_list(&p);
  p_ws(&p);
  if (!p_eof(&p)) {
    if (status) *status = 1;
    if (err && errlen) {
      size_t fp = p.fail_pos > p.pos ? p.fail_pos : p.pos;
      int line = 1; for (size_t i = 0; i < fp && i < p.n; ++i) if (text[i] == '\n') line++;
      snprintf(err, (size_t)errlen, "parse error near line %d (offset %zu)", line, fp);
    }
    return sc;
  }
  if (p.unimplemented) {          /* AstStatement::from_pest panics before anything executes */
    if (err && errlen) snprintf(err, (size_t)errlen, "not implemented: command '%s'", p.unimplemented);
    if (status) *status = 2;
    orc_free_scene(sc);
    return NULL;
  }
  Ctx c;
  memset(&c, 0, sizeof c);
  c.sc = sc;
  Value tv; memset(&tv, 0, sizeof tv);
  tv.kind = V_NUMBER; tv.num = time;
  map_insert(&c, &c.globals, "time", tv);                                           /* scene_loader.rs:34 */
  exec(&c, ast);
  free(c.stack);
  if (c.failed) {
    if (err && errlen) snprintf(err, (size_t)errlen, "%s", c.err);
    if (status) *status = 2;
    orc_free_scene(sc);
    return NULL;
  }
  return sc;
}

void orc_set_max_depth(orc_scene *sc, int d) { sc->max_depth = d; }
int orc_num_objects(const orc_scene *sc) { return sc->n_objects; }
int orc_num_lights(const orc_scene *sc) { return sc->n_lights; }
void orc_camera(const orc_scene *sc, double out[10]) {
  const Camera *c = &sc->camera;
  out[0] = c->center.x; out[1] = c->center.y; out[2] = c->center.z;
  out[3] = c->direction.x; out[4] = c->direction.y; out[5] = c->direction.z;
  out[6] = c->right.x; out[7] = c->right.y; out[8] = c->right.z;
  out[9] = c->aspect_ratio;
}
void orc_light(const orc_scene *sc, int i, double out[7]) {
  const PointLight *l = &sc->lights[i];
  out[0] = l->point.x; out[1] = l->point.y; out[2] = l->point.z;
  out[3] = l->color.r; out[4] = l->color.g; out[5] = l->color.b; out[6] = l->color.a;
}

void orc_get_pixel(const orc_scene *sc, double x, double y, double rgba[4]) {
  Color col = get_pixel(sc, x, y);
  rgba[0] = col.r; rgba[1] = col.g; rgba[2] = col.b; rgba[3] = col.a;
}

/* Texel-boundary probe (tests only): the primary ray of get_pixel(x, y) (camera.rs:58-74), its nearest
 * hit (raytracer.rs:141-150) and, when the hit object is textured, the texture lookup's coordinates
 * before truncation (texture.rs:27-34): out = {u * (w - 1), h - v * (h - 1) - 1, u, v}.  Returns the
 * hit object's index if it is textured, else -1. */
int orc_texel_probe(const orc_scene *sc, double x, double y, double out[4]) {
  Ray ray = camera_create_ray(&sc->camera, x, y);
  NearestCtx nc = {INFINITY, NULL, NULL};
  for (int i = 0; i < sc->n_objects; ++i) {
    nc.cur = &sc->objects[i];
    rtobject_intersects(&sc->objects[i], ray, add_nearest, &nc);
  }
  const RTObject *obj = nc.nearest_obj;
  if (!obj || !obj->material.textured) return -1;
  Vec point = v_add(ray.point, v_scale(ray.direction, nc.nearest));
  UV uv = {0.0, 0.0};
  if (!shape_get_uv(obj->shape, point, &uv)) { uv.u = 0.0; uv.v = 0.0; }
  const Texture *t = obj->material.texture;
  out[0] = uv.u * (double)(t->w - 1);
  out[1] = (double)t->h - (uv.v * (double)(t->h - 1)) - 1.0;
  out[2] = uv.u;
  out[3] = uv.v;
  return (int)(obj - sc->objects);
}

/* Test infrastructure: get_pixel(x, y)'s primary hit (raytracer.rs:138-150) and, for each light, whether its
 * shadow ray is occluded (transparency != 1, raytracer.rs:176-197) -- the signature whose changes along a
 * scan line are the frame's silhouettes and shadow edges (tests/test_gpu_cull_edges.py bisects them).
 * Returns -1 on a miss, else object + 1 + 4096 * (bit i: light i occluded); *t = the hit distance. */
long long orc_hit_signature(const orc_scene *sc, double x, double y, double *t) {
  Ray ray = camera_create_ray(&sc->camera, x, y);
  NearestCtx nc = {INFINITY, NULL, NULL};
  for (int i = 0; i < sc->n_objects; ++i) {
    nc.cur = &sc->objects[i];
    rtobject_intersects(&sc->objects[i], ray, add_nearest, &nc);
  }
  *t = nc.nearest;
  if (!nc.nearest_obj) return -1;
  Vec point = v_add(ray.point, v_scale(ray.direction, nc.nearest));
  long long mask = 0;
  for (int li = 0; li < sc->n_lights && li < 40; ++li) {
    const PointLight *light = &sc->lights[li];
    Ray shadow_ray;
    shadow_ray.point = point;
    shadow_ray.direction = v_normalized(v_sub(light->point, point));
    ShadowCtx sh;
    sh.distance = v_length(v_sub(light->point, point));
    sh.transparency = 1.0;
    sh.uv.u = sh.uv.v = 0.0;
    for (int i = 0; i < sc->n_objects; ++i) {
      sh.cached = &sc->objects[i];
      rtobject_intersects(&sc->objects[i], shadow_ray, add_shadow, &sh);
    }
    if (sh.transparency != 1.0) mask |= 1ll << li;
  }
  return (long long)(nc.nearest_obj - sc->objects) + 1 + 4096 * mask;
}

typedef struct {
  const orc_scene *sc;
  int y0, y1, tid, nthreads, row_step;
  double *f64; uint8_t *u8;
  uint64_t cnt[C_NUM];
} Job;

static void *render_job(void *vj) {
  Job *j = (Job *)vj;
  const orc_scene *sc = j->sc;
  int W = sc->width;
#if ORC_COUNTERS
  memset(j->cnt, 0, sizeof j->cnt);
  g_cnt = j->cnt;
#endif
  /* rows interleaved across threads (the reference's threadpool is sized to num_cpus) */
  int k = 0;
  for (int y = j->y0; y < j->y1; y += j->row_step, ++k) {
    if (k % j->nthreads != j->tid) continue;
    size_t row = (size_t)k;   /* output row index */
    for (int x = 0; x < W; ++x) {                                                   /* debug_window.rs:74-87 */
      Color col = get_pixel(sc, (double)x, (double)y);
      size_t o = (row * (size_t)W + (size_t)x) * 4;
      if (j->f64) { j->f64[o] = col.r; j->f64[o + 1] = col.g; j->f64[o + 2] = col.b; j->f64[o + 3] = col.a; }
      if (j->u8) { j->u8[o] = to_u8(col.r); j->u8[o + 1] = to_u8(col.g); j->u8[o + 2] = to_u8(col.b); j->u8[o + 3] = to_u8(col.a); }
    }
  }
  return NULL;
}

/* Render rows y0, y0+step, ... < y1 (step >= 1) into packed output rows. Either
 * output may be NULL.  counters (may be NULL) receives C_NUM event counts (counting build). */
int orc_render_rows(const orc_scene *sc, int y0, int y1, int row_step, double *f64, uint8_t *u8,
                    int nthreads, uint64_t *counters) {
  if (nthreads < 1) nthreads = 1;
  if (row_step < 1) row_step = 1;
  Job *jobs = (Job *)calloc((size_t)nthreads, sizeof(Job));
  pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; ++t) {
    jobs[t].sc = sc; jobs[t].y0 = y0; jobs[t].y1 = y1; jobs[t].tid = t; jobs[t].nthreads = nthreads;
    jobs[t].row_step = row_step; jobs[t].f64 = f64; jobs[t].u8 = u8;
  }
  if (nthreads == 1) render_job(&jobs[0]);
  else {
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, render_job, &jobs[t]);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  }
  if (counters) {
    memset(counters, 0, sizeof(uint64_t) * C_NUM);
    for (int t = 0; t < nthreads; ++t)
      for (int e = 0; e < C_NUM; ++e) counters[e] += jobs[t].cnt[e];
  }
  free(jobs); free(th);
  return 0;
}

int orc_num_counters(void) { return C_NUM; }
int orc_counting_build(void) { return ORC_COUNTERS; }

/* ------------------------------------------------------------------------- */
/* Adaptive anti-aliasing (antialiaser.rs), restated depth-first with the     */
/* reference's per-pixel memo grid.  Input = the QUANTISED frame re-read as   */
/* u8/255 colours (debug_window.rs:280-286, easy_pixbuf.rs:55-64).            */
/* ------------------------------------------------------------------------- */
typedef struct {
  const orc_scene *sc;
  const uint8_t *src; size_t stride;
  double threshold; int level, size;
  int x, y;
  Color *grid; unsigned char *have;     /* sub_pixels[sub_x][sub_y]: Option<Color> */
  uint64_t rays;
} AaPixel;

static Color aa_src(const AaPixel *a, int x, int y) {                 /* easy_pixbuf.rs:55-64 */
  const uint8_t *p = a->src + (size_t)y * a->stride + (size_t)x * 4;
  Color c = {p[0] / 255.0, p[1] / 255.0, p[2] / 255.0, p[3] / 255.0};
  return c;
}

static int aa_different(Color c1, Color c2, double threshold) {         /* antialiaser.rs:154-162 */
  return (fabs(c1.r - c2.r) + fabs(c1.g - c2.g) + fabs(c1.b - c2.b) + fabs(c1.a - c2.a)) / 4.0 > threshold;
}

static Color aa_average(Color c1, Color c2, Color c3, Color c4) {      /* antialiaser.rs:164-171 */
  Color c = {(c1.r + c2.r + c3.r + c4.r) / 4.0, (c1.g + c2.g + c3.g + c4.g) / 4.0,
             (c1.b + c2.b + c3.b + c4.b) / 4.0, (c1.a + c2.a + c3.a + c4.a) / 4.0};
  return c;
}

static Color aa_sub(AaPixel *a, int sx, int sy) {                       /* antialiaser.rs:101-115 */
  int i = sx * a->size + sy;
  if (a->have[i]) return a->grid[i];
  a->rays++;
  Color c = get_pixel(a->sc, (double)a->x + ((double)sx / (double)a->size),
                      (double)a->y + ((double)sy / (double)a->size));
  a->grid[i] = c; a->have[i] = 1;
  return c;
}

static Color aa_cell(AaPixel *a, int x1, int y1, int x2, int y2, int level) {   /* antialiaser.rs:124-152 */
  Color c1 = aa_sub(a, x1, y1), c2 = aa_sub(a, x2, y1), c3 = aa_sub(a, x1, y2), c4 = aa_sub(a, x2, y2);
  int different = aa_different(c1, c2, a->threshold) || aa_different(c1, c3, a->threshold) ||
                  aa_different(c1, c4, a->threshold);
  if (!different || level <= 0) return aa_average(c1, c2, c3, c4);
  int mx = x1 + (x2 - x1) / 2, my = y1 + (y2 - y1) / 2;
  Color d1 = aa_cell(a, x1, y1, mx, my, level - 1);
  Color d2 = aa_cell(a, mx, y1, x2, my, level - 1);
  Color d3 = aa_cell(a, x1, my, mx, y2, level - 1);
  Color d4 = aa_cell(a, mx, my, x2, y2, level - 1);
  return aa_average(d1, d2, d3, d4);
}

typedef struct {
  const orc_scene *sc; const uint8_t *src; size_t stride; double threshold; int level;
  int tid, nthreads; double *f64; uint8_t *u8; uint64_t rays;
} AaJob;

static void aa_put(AaJob *j, int x, int y, Color c) {
  size_t o = ((size_t)y * (size_t)j->sc->width + (size_t)x) * 4;
  if (j->f64) { j->f64[o] = c.r; j->f64[o + 1] = c.g; j->f64[o + 2] = c.b; j->f64[o + 3] = c.a; }
  if (j->u8) { j->u8[o] = to_u8(c.r); j->u8[o + 1] = to_u8(c.g); j->u8[o + 2] = to_u8(c.b); j->u8[o + 3] = to_u8(c.a); }
}

static void *aa_job(void *vj) {
  AaJob *j = (AaJob *)vj;
  const int W = j->sc->width, H = j->sc->height;
  AaPixel a;
  memset(&a, 0, sizeof a);
  a.sc = j->sc; a.src = j->src; a.stride = j->stride; a.threshold = j->threshold; a.level = j->level;
  a.size = (1 << j->level) + 1;                                          /* antialiaser.rs:20 */
  a.grid = (Color *)malloc(sizeof(Color) * (size_t)a.size * (size_t)a.size);
  a.have = (unsigned char *)malloc((size_t)a.size * (size_t)a.size);
  for (int y = 0; y < H; ++y) {
    if (y % j->nthreads != j->tid) continue;
    if (y == H - 1) {                  /* debug_window.rs:298: the AA pass never touches the last row */
      for (int x = 0; x < W; ++x) aa_put(j, x, y, aa_src(&a, x, y));
      continue;
    }
    for (int x = 0; x < W - 1; ++x) {                                    /* antialiaser.rs:53-71 */
      const int n = a.size - 1;
      memset(a.have, 0, (size_t)a.size * (size_t)a.size);                /* clear_matrices */
      a.x = x; a.y = y;
      a.grid[0] = aa_src(&a, x, y);                 a.have[0] = 1;        /* :96-99 */
      a.grid[0 * a.size + n] = aa_src(&a, x, y + 1); a.have[0 * a.size + n] = 1;
      a.grid[n * a.size + 0] = aa_src(&a, x + 1, y); a.have[n * a.size + 0] = 1;
      a.grid[n * a.size + n] = aa_src(&a, x + 1, y + 1); a.have[n * a.size + n] = 1;
      aa_put(j, x, y, aa_cell(&a, 0, 0, n, n, j->level));
    }
    aa_put(j, W - 1, y, aa_src(&a, W - 1, y));                          /* copy the last pixel */
  }
  j->rays = a.rays;
  free(a.grid); free(a.have);
  return NULL;
}

/* Anti-alias a whole quantised frame (RGBA8, row stride `stride` bytes) of the scene's size.
 * Outputs (either may be NULL) are full frames; the last row and column are the source pixels
 * re-quantised.  Returns the number of sub-pixel rays traced (the reference's ray_counter). */
long long orc_antialias(const orc_scene *sc, const uint8_t *src, size_t stride, double threshold,
                        int level, double *f64, uint8_t *u8, int nthreads) {
  if (level < 0) level = 0;
  if (level > 12) return -1;
  if (nthreads < 1) nthreads = 1;
  AaJob *jobs = (AaJob *)calloc((size_t)nthreads, sizeof(AaJob));
  pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; ++t) {
    jobs[t].sc = sc; jobs[t].src = src; jobs[t].stride = stride; jobs[t].threshold = threshold;
    jobs[t].level = level; jobs[t].tid = t; jobs[t].nthreads = nthreads; jobs[t].f64 = f64; jobs[t].u8 = u8;
  }
  if (nthreads == 1) aa_job(&jobs[0]);
  else {
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, aa_job, &jobs[t]);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  }
  long long rays = 0;
  for (int t = 0; t < nthreads; ++t) rays += (long long)jobs[t].rays;
  free(jobs); free(th);
  return rays;
}

/* ------------------------------------------------------------------------- */
/* Orthogonal preview views (debug_window.rs:166-227, ray_debugger.rs:33-68). */
/* ------------------------------------------------------------------------- */
typedef struct { double distance; const RTObject *foremost, *cur; } OrthoCtx;
static void add_ortho(void *vctx, double d) {                                      /* debug_window.rs:205-210 */
  OrthoCtx *c = (OrthoCtx *)vctx;
  if (d < c->distance) { c->foremost = c->cur; c->distance = d; }
}

static double *vaxis(Vec *v, int a) { return a == 0 ? &v->x : (a == 1 ? &v->y : &v->z); }

/* Rows [y0, y1) of an orthogonal view at the scene's W x H: flat RTObject::get_color
 * (rt_object.rs:45-47) of the object with the smallest intersection distance (any sign, no EPS),
 * Color::EMPTY on a miss.  Returns -1 for invalid axes (the reference panics). */
int orc_render_ortho(const orc_scene *sc, int axis1, int axis2, double dir1, double dir2, double scale,
                     int y0, int y1, double *f64, uint8_t *u8) {
  const int W = sc->width, H = sc->height;
  const double center_x = (double)W / 2.0, center_y = (double)H / 2.0;
  int axis3;
  if (axis1 < 0 || axis1 > 2 || axis2 < 0 || axis2 > 2) return -1;
  if (axis1 != 0 && axis2 != 0) axis3 = 0;
  else if (axis1 != 1 && axis2 != 1) axis3 = 1;
  else if (axis1 != 2 && axis2 != 2) axis3 = 2;
  else return -1;                                                                  /* panic!("Invalid axes") */
  Vec direction = {0.0, 0.0, 0.0};
  *vaxis(&direction, axis3) = 1.0;
  (void)H;
  for (int y = y0; y < y1; ++y) {
    for (int x = 0; x < W; ++x) {
      Ray ray;
      ray.point.x = ray.point.y = ray.point.z = 0.0;
      *vaxis(&ray.point, axis1) = (((double)x - center_x) * dir1) / scale;
      *vaxis(&ray.point, axis2) = (((double)y - center_y) * dir2) / scale;
      *vaxis(&ray.point, axis3) = 10000.0;
      ray.direction = direction;
      OrthoCtx oc = {INFINITY, NULL, NULL};
      for (int i = 0; i < sc->n_objects; ++i) {
        oc.cur = &sc->objects[i];
        rtobject_intersects(&sc->objects[i], ray, add_ortho, &oc);
      }
      Color c = {0.0, 0.0, 0.0, 0.0};                                              /* Color::EMPTY */
      if (oc.foremost) {
        const Material *m = &oc.foremost->material;
        if (m->textured) { UV uv = {0.0, 0.0}; c = texture_color_at(m->texture, uv); }
        else c = m->color;
      }
      size_t o = ((size_t)(y - y0) * (size_t)W + (size_t)x) * 4;
      if (f64) { f64[o] = c.r; f64[o + 1] = c.g; f64[o + 2] = c.b; f64[o + 3] = c.a; }
      if (u8) { u8[o] = to_u8(c.r); u8[o + 1] = to_u8(c.g); u8[o + 2] = to_u8(c.b); u8[o + 3] = to_u8(c.a); }
    }
  }
  return 0;
}

/* RayDebugger::record_rays (ray_debugger.rs:92-137): the rays of pixel (x, y) in callback order.
 * Returns the number of rays (records beyond cap are dropped); rgba = get_pixel's colour. */
int orc_record_rays(const orc_scene *sc, double x, double y, OrcRayRecord *out, int cap, double rgba[4]) {
  OrcRec r = {sc, out, cap, 0};
  g_rec = &r;
  Color c = get_pixel(sc, x, y);
  g_rec = NULL;
  rgba[0] = c.r; rgba[1] = c.g; rgba[2] = c.b; rgba[3] = c.a;
  return r.n;
}
int orc_ray_record_size(void) { return (int)sizeof(OrcRayRecord); }
