// rt_blob.h -- the flattened, immutable scene as it lives in HBM (shared by the host
// flattener, scene.cpp, and the gfx950 kernels, rt_device.h).
//
// Design (DESIGN.md "Data layout in HBM"):
//  * The reference walks a tree of boxed trait objects per ray (RTObject -> dyn MathShape
//    -> CSG -> RTObject ...).  Here every top-level object is flattened once on the host into
//      - a contiguous run of RtNode in POST-ORDER (children before parents, root last), used
//        to evaluate CSG is_inside / is_on_surface bottom-up at a shaded point;
//      - a contiguous run of RtLeaf (the primitives, DFS order), each carrying everything the
//        reference recomputes per call (inverse-origin, normalised plane normal, r*r, r+EPS,
//        cube slab bounds, the six cube "quirk" planes and their transformed normals), computed
//        on the host with the IDENTICAL f64 op sequence so the device reads bit-equal values;
//      - per leaf, a tiny postfix "hit filter" program: the conjunction of the sibling
//        is_inside tests every CSG ancestor applies to a hit of that leaf (csg.rs:39-96).
//  * All indices into these arrays are wave-uniform in the kernels (every lane walks the same
//    object list), so the loads compile to scalar (SMEM) loads through the scalar cache.
//  * Textures stay RGBA8 in HBM (the reference holds f64 RGBA, 32 B/texel); the kernel
//    converts with /255.0 exactly as sceneparser/texture.rs:29-33 does.
#pragma once
#ifndef __HIPCC_RTC__
#include <stdint.h>
#else                                // hipRTC (spec.hip): its runtime header keeps these in a namespace
using __hip_internal::int32_t;
using __hip_internal::int64_t;
using __hip_internal::uint8_t;
using __hip_internal::uint32_t;
using __hip_internal::uint64_t;
#endif

#define RT_EPSILON 10e-7            /* math.rs:2 */
#define RT_CULL_COORD_MAX 1e6        /* culling boxes / ray origins beyond this are never culled */
/* f32 culling (rt_device.h fbox_may_hit): rays whose origin has a coordinate beyond RT_CULL32_COORD_MAX
 * are never culled; every f32 box is the f64 box grown by RT_CULL32_MARGIN = RT_CULL32_COORD_MAX * 2^-22
 * (4x the rounding of an origin coordinate to f32) and then rounded outward to f32 (scene.cpp). */
#define RT_CULL32_COORD_MAX 65536.0
#define RT_CULL32_MARGIN (RT_CULL32_COORD_MAX / 4194304.0)
#define RT_MAX_DEPTH_CAP 16          /* recursion frames kept per lane (max_depth <= 16) */
#define RT_MAX_LITS 4                /* inline hit-filter literals per leaf */

// Kernel modes (rt_device.h trace, k_rows.hip): the reflection-only megakernel; refraction scenes
// whose rays form chains (RtDevScene::ray_chains); refraction scenes with ray trees.
// Pixel tile of one wave: RT_TILE_W x (64 / RT_TILE_W) pixels (rt_device.h tile_pixel).  8 x 8 by
// default; diagnostic builds may set 16 (16 x 4) or 32 (32 x 2).
#ifndef RT_TILE_W
#define RT_TILE_W 8
#endif
#define RT_MODE_REFL 0
#define RT_MODE_CHAIN 1
#define RT_MODE_TREE 2

enum RtNodeKind : int32_t {
  RT_N_SPHERE = 0, RT_N_PLANE = 1, RT_N_CUBE = 2,
  RT_N_UNION = 3, RT_N_INTERSECTION = 4, RT_N_DIFFERENCE = 5
};

// Conservative culling bounds (world-space AABB of every point where an ACCEPTED hit of the
// leaf / object can lie, inflated far beyond f64 rounding).  They only skip work whose result
// cannot be used: the rendered bits are unchanged (DESIGN.md "Culling").
enum RtCull : int32_t {
  RT_CULL_NONE = 0,     // unbounded (planes, singular transforms): always evaluate
  RT_CULL_BOX = 1,      // test the ray segment against [blo, bhi]
  RT_CULL_ALWAYS = 2,   // provably no accepted hit (empty CSG intersection)
};

// Hit-filter program opcodes (postfix over a bit stack).
enum RtProgOp : int32_t {
  RT_OP_INSIDE = 0,     // push leaf[arg].is_inside(p)
  RT_OP_AND = 1,        // a && b
  RT_OP_OR = 2,         // a || b
  RT_OP_ANDNOT = 3,     // a && !b
  RT_OP_REQUIRE = 4,    // pop v; filter &= (v == arg)
};

struct RtProg { int32_t op, arg; };

#define RT_XF_IDENTITY 2   // RtLeaf::xdiag value of an identity inverse (a diagonal-affine special case)

struct alignas(16) RtLeaf {
  // Field order = access order of a traversal's leaf evaluation (the kernels read these through
  // scalar loads, 64-byte scalar-cache lines): the integer header and the culling box, then the
  // inverse transform, then the primitive's parameters; the shading-only fields (forward matrix,
  // surface tests, quirk planes) last.
  int32_t kind;         // RtNodeKind (leaf kinds only)
  int32_t cull;         // RtCull
  int32_t xdiag;        // 1: inv is diagonal-affine (see below): transform_vector has a 2-op form;
                        // RT_XF_IDENTITY: inv is the identity and inv_o = 0: no transform at all
  int32_t share_prev;   // sphere leaf: 1 = the previous leaf of the object is a sphere with a bit-identical
                        // inverse transform (inv, inv_o, xdiag) and centre, and every traversal that
                        // evaluates this leaf has evaluated that one first (see below)
  int32_t plane_axis;   // untransformed plane leaf: 0/1/2 when pnorm has exactly one nonzero (finite) component; else -1
  int32_t filter_const; // 1: every literal of the hit filter passes for any hit of this leaf whose ray origin is
                        // within 1e6 (concentric spheres under one transform, radii apart by more than the
                        // rounding margin: scene.cpp const_filters), so the traversals skip the filter
  int32_t prog_begin;   // hit-filter program [prog_begin, prog_end)
  int32_t prog_end;
  int32_t n_lit;        // >= 0: the filter program is the conjunction of n_lit literals below
  int32_t lit[RT_MAX_LITS];   // literal = 2 * leaf + want: leaf[lit >> 1].is_inside(p) == (lit & 1)
  int32_t object;       // the top-level object this leaf belongs to (the cooperative tail walk, rt_device.h)
  int32_t pad0[2];
  float fblo[3], fbhi[3]; // blo / bhi as the f32 culling box (RT_CULL32_MARGIN, rounded outward)
  int32_t pad1[2];
  double blo[3], bhi[3];// culling box of this leaf's accepted hits (own bound ^ required-inside siblings)
  double inv[12];       // inverse matrix rows 0..2 (row-major, 4 per row)
  double inv_o[3];      // transform_vector((0,0,0), inverse)   (transformation.rs:80-83)
  double c[3];          // sphere / cube centre
  double radius;        // sphere radius | cube half length ("length", math_shapes.rs:229)
  double r2;            // sphere: radius * radius
  double r_eps;         // sphere: radius + EPSILON
  double lo[3];         // cube: centre - length
  double hi[3];         // cube: centre + length
  double pnorm[3];      // plane leaf: Vector::new(a,b,c).normalized() (math_shapes.rs:169)
  double pl[6][4];      // plane leaf: pl[0] = raw (a,b,c,d); cube: p1..p6 raw (a,b,c,d)
  double lo_e[3];       // cube: centre - length - EPSILON
  double hi_e[3];       // cube: centre + length + EPSILON
  double mat[12];       // forward matrix rows 0..2
  double mat_o[3];      // transform_vector((0,0,0), matrix)    (transformation.rs:71-74)
  double pn[6][3];      // matching transformed unit normals (MathPlane::normal)
};
// share_prev: the traversals evaluate an object's leaves in order, each unless its own box test
// culls it (only when the object has leaf_cull).  The host sets share_prev only if the previous
// leaf is never skipped when this one is evaluated: the object has no per-leaf culling, or the
// previous leaf's cull is NONE, or both are BOX tests with this leaf's box inside the previous
// one's.  The box test's slab times are monotone in the bounds and tmax never grows along the
// loop, so a ray that passes the inner box has passed the outer one.
// plane_axis = a: dot(pnorm, v) = (n0*v.x + n1*v.y) + n2*v.z equals n_a * v_a for FINITE v whenever
// n_a * v_a != 0 (the other two products are signed zeros); when n_a * v_a is +-0 the sum is some
// +-0 too.  The plane test only asks `v_d != 0` of the direction term and, for traversals (t > EPS
// wanted), the strict signs of num = dot(pnorm, o) + d and v_d, which a signed zero never passes,
// so the short form decides every traversal test exactly (rt_device.h leaf_candidates).
// Literal form: most CSG filters (every ancestor requiring an intersection / difference sibling
// inside, or a union sibling outside) are a plain conjunction of single-leaf is_inside tests;
// the host rewrites the postfix program into at most RT_MAX_LITS literals (n_lit = -1: keep the
// program).  The tests are pure, so their order is free.
// xdiag: the inverse's 3x3 part is diagonal (off-diagonal entries are +-0) and every entry is
// finite.  For FINITE inputs transform_vector's row ((m00*x + m01*y) + m02*z) + m03 then equals
// m00*x + m03 except possibly in the SIGN of an exactly-zero result (the dropped terms are
// signed zeros: they leave any nonzero partial sum unchanged).  No consumer can observe that
// sign: object-space points and directions only reach comparisons, fabs, squares and sums with
// the other components; a zero distance is rejected by `d > EPS` (and compares equal either way
// in the ortho views); a zero direction component takes the `dir == 0` branch of the cube slab
// test for both signs.  The kernel takes the short form only when every input of the wave is
// finite (0 * inf would be NaN in the full form).  RT_XF_IDENTITY (diagonal entries exactly 1,
// translations and inv_o exactly +-0) is the same argument once more: 1 * x + (+-0) = x up to the
// sign of a zero, and a direction minus inv_o = +-0 likewise, so the transform is skipped.

struct RtNode {
  int32_t kind;         // RtNodeKind
  int32_t a, b;         // CSG children: node indices relative to the object's node_begin
  int32_t leaf;         // leaf kinds: global leaf index
};

struct alignas(16) RtObject {
  int32_t node_begin, node_count;   // post-order; root = node_begin + node_count - 1
  int32_t leaf_begin, leaf_count;
  int32_t textured;                 // 0 solid, 1 texture
  int32_t tex;                      // texture index
  int32_t shadow_skip;              // transparency == 1.0: shadow multiplies by 1 -> no-op
  int32_t cull;                     // RtCull for the object box (hull of its leaves' boxes)
  double color[3];                  // material colour (solid)
  double color_a;                   // its alpha (only the ortho views read it)
  double reflectivity, transparency;
  double blo[3], bhi[3];
  int32_t leaf_cull;                // 1: per-leaf boxes are tighter than the object box
  int32_t obb_leaf;                 // >= 0: every accepted hit of the object lies inside this leaf's
                                    // region, whose box in the leaf's OWN frame (olo, ohi) is much
                                    // tighter than blo/bhi (rotated thin rods and slabs); -1: none
  double olo[3], ohi[3];            // that box in obb_leaf's object space, inflated (scene.cpp obb)
  float folo[3], fohi[3];           // olo / ohi as the f32 culling box (RT_CULL32_MARGIN, rounded outward)
  int32_t unit_normal;              // 1: the normal is a constant (a plane object): nunit / nunit_len below
  int32_t pad1;
  double nunit[3];                  // normalized(get_normal) (raytracer.rs:163), the host's IEEE operations
  double nunit_len;                 // len(nunit) (vector.rs:57-59's denominator term)
};

// Order-preserving object hierarchy: a pre-order list of nodes over CONTIGUOUS runs of objects
// in draw order.  A group node's box is the hull of its objects' boxes; a ray that misses it
// skips to `skip`.  Objects are still visited in increasing index order, so the nearest-hit tie
// rule (first object wins) and the shadow product order are the reference's.
struct alignas(16) RtTrav {
  double blo[3], bhi[3];            // group: hull of its objects' boxes; object node: a copy of the object's box
  int32_t obj;                      // >= 0: object index; -1: group node
  int32_t skip;                     // node index after this node's subtree
  int32_t cull;                     // object node: a copy of RtObject::cull (one record per step of a
  int32_t shadow_skip;              //   per-lane walk, k_wavefront.hip wfp_cand_kernel), ::shadow_skip
  float fblo[3], fbhi[3];           // blo / bhi as the f32 culling box (RT_CULL32_MARGIN, rounded outward)
  int32_t pad0[2];
};

// A hierarchy node in the form the generic kernels' walks read (rt_device.h walk_trav: one node per step,
// a dependent scalar load; the wavefront path's per-lane walk, staged in LDS): 32 B instead of RtTrav's
// 96 -- the f32 culling box and the node words, cull and shadow_skip packed above the 28-bit skip -- two
// nodes per 64-byte scalar-cache line.  (RtTrav's f32 box sits past its first line: fractal.scene's
// 300-node walks read two lines per step and its wavefront level-0 trace ran 2.9x longer.)
struct alignas(16) RtTravC {
  float lo[3], hi[3];               // RtTrav::fblo / fbhi
  int32_t obj;                      // RtTrav::obj
  uint32_t skip_flags;              // skip | cull << 28 | shadow_skip << 30
};

struct RtTexture {
  int64_t offset;                   // byte offset of RGBA8 data in the texel pool
  int32_t w, h;
};

struct RtLight { double p[3]; double col[3]; };

struct RtCamera {
  double center[3], direction[3], right[3], up[3];
  double aspect, width, height;     // as f64: `self.width as f64` (camera.rs:67-68)
};

// Kernel argument block (passed by value; all pointers are device pointers).
struct RtDevScene {
  const RtObject* objects;
  const RtTrav* trav;
  const RtTrav* strav;              // shadow rays of scenes without a transparent object (any order is exact)
  const RtTravC* trav_c;            // trav and strav, compact (the generic kernels' walks, the wavefront walk)
  const RtTravC* strav_c;
  const RtNode* nodes;
  const RtLeaf* leaves;
  const RtProg* prog;
  const RtLight* lights;
  const RtTexture* textures;
  const uint8_t* texels;
  int32_t n_objects, n_lights, n_leaves, n_nodes, n_trav, n_strav;
  int32_t width, height;
  int32_t any_transparent;          // some object has transparency != 0 (refraction possible)
  int32_t shadow_early_out;         // every transparency is finite: product==0 stays 0
  int32_t colour_fast;              // colour clamps may take the min/max form (rt_device.h FC)
  int32_t ray_chains;               // every hit spawns at most one ray (scene.cpp flatten)
  int32_t shadow_pow;               // a shadow product depends only on its factors' multiset: every
                                    // transparency is finite and all those other than +-0 and 1 are
                                    // one value, shadow_t (scene.cpp flatten; the wavefront pair path)
  double shadow_t;
  RtCamera cam;
  // get_pixel(x as f64, y as f64)'s per-column and per-row camera terms for integer pixels (rt_ctx
  // upload, the host's IEEE evaluation of camera_ray's own expressions): width and height doubles
  const double* cam_sx;
  const double* cam_sy;
};
