// scene.h -- host-side scene model behind the C ABI (rt_scene) and its flattener.
//
// rt_scene mirrors the reference's RayTracer after the scene parser filled it
// (raytracer.rs:21-35): a list of top-level objects (shape tree + material), point lights,
// a camera centre and max_depth.  Shapes are immutable value records addressed by id; the
// device layout (rt_blob.h) is produced by rt::flatten at upload time.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/rt_abi.h"
#include "rt_blob.h"

namespace rt {

// Thread-local last error (rt_last_error).  Returns `status` so call sites can
// `return fail(RT_ERR_INVALID, "...")`.
int fail(int status, const char* fmt, ...);
void set_error_message(const std::string& msg);

enum ShapeKind : int32_t { SHAPE_SPHERE = 0, SHAPE_PLANE = 1, SHAPE_CUBE = 2, SHAPE_CSG = 3 };

struct ShapeRec {
  ShapeKind kind;
  rt_transformation t;      // leaves: the shape's MatrixTransformation
  double center[3];         // sphere / cube centre
  double size;              // sphere radius | cube edge length (before the /2 of MathCube::new)
  double normal[3];         // plane (a, b, c)
  double distance;          // plane d
  rt_csg_op op;             // CSG
  int32_t a, b;             // CSG children (shape ids)
};

struct ObjectRec { int32_t shape; rt_material mat; };
struct LightRec { double p[3]; double color[4]; double fade; };
struct TextureRec { uint32_t w, h; std::vector<uint8_t> rgba; };

// Flattened scene, host copy of what goes to HBM.
struct FlatScene {
  std::vector<RtObject> objects;
  std::vector<RtTrav> trav;
  std::vector<RtTrav> strav;       // shadow-ray hierarchy: likeliest occluders first (scene.cpp build_hierarchy)
  std::vector<RtNode> nodes;
  std::vector<RtLeaf> leaves;
  std::vector<RtProg> prog;
  std::vector<RtLight> lights;
  std::vector<RtTexture> textures;
  std::vector<uint8_t> texels;
  RtCamera cam;
  int32_t width, height, max_depth;
  int32_t any_transparent, shadow_early_out;
  int32_t colour_fast;   // every colour-op operand is finite and >= +0 (see flatten)
  int32_t ray_chains;    // every hit spawns at most one ray: no object is both transparent and reflective
  int32_t shadow_pow;    // shadow products are order-free (see RtDevScene::shadow_pow)
  double shadow_t;
};

// Transformation math (transformation.rs:104-220), exact f64 op order.
void xf_identity(rt_transformation* t);
void xf_translation(double x, double y, double z, rt_transformation* t);
void xf_rotation(double x, double y, double z, rt_transformation* t);
void xf_scaling(double x, double y, double z, rt_transformation* t);
void xf_compose(const rt_transformation& self, const rt_transformation& other, rt_transformation* out);
void xf_apply(const double m[16], const double v[3], double out[3]);   // transform_vector

}  // namespace rt

struct rt_scene {
  uint32_t width = 0, height = 0;
  int32_t max_depth = 10;
  double cam_center[3] = {0.0, 0.0, -100.0};
  std::vector<rt::ShapeRec> shapes;
  std::vector<rt::ObjectRec> objects;
  std::vector<rt::LightRec> lights;
  std::vector<rt::TextureRec> textures;
};

namespace rt {
int flatten(const rt_scene& s, FlatScene* out);
std::string describe_flat(const FlatScene& f);   // rt_scene_describe's text
// A diagnostic switch from the environment: only in a diagnostic build (make diag DIAG=-DRT_DIAG_ENV),
// false in the product (rt_ctx.hip).
bool diag_env(const char* name);
// DSL front end (scene_dsl.cpp): fills a fresh default scene.
int compile_scene_text(const char* text, const char* asset_dir, double time, rt_scene* scene);
// PNG (png_io.cpp)
int png_decode_rgba8(const std::vector<uint8_t>& file, std::vector<uint8_t>* rgba, uint32_t* w, uint32_t* h);
int png_encode(const uint8_t* rgba8, uint32_t w, uint32_t h, size_t stride, int channels,
               std::vector<uint8_t>* out);
bool read_file(const std::string& path, std::vector<uint8_t>* out);
}  // namespace rt
