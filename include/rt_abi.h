/*
 * rt_abi.h -- C ABI of the MI355X-native TinyRaytracer render path (librt_mi355x.so).
 *
 * This is the drop-in seam for the reference's src/raytracer render loop
 * (andreivasiliu/TinyRaytracerInRust).  The reference has no FFI; its seam is the
 * `RayTracer` the scene parser fills and the GUI worker renders row by row.  Each
 * entry point below names the reference interface it replaces (file:line under
 * src/).  The Rust-side `extern "C"` block a maintainer would add is shown in
 * INTEGRATION.md.
 *
 * Conventions
 *   - every function returns RT_OK (0) or a negative rt_status; none aborts (one exception:
 *     rt_ctx_spec_wait returns RT_PENDING (> 0) when its time limit passes first);
 *     rt_last_error() returns a thread-local message for the last failure;
 *   - no torch / HIP types in signatures: plain pointers, sizes and an opaque
 *     `void* stream` (a hipStream_t; NULL = the device's default stream, as in HIP);
 *   - the library owns rt_scene / rt_ctx; the caller owns every output buffer;
 *   - an rt_scene is immutable once uploaded and may be shared by threads; an
 *     rt_ctx is used by one host thread at a time; distinct contexts may run
 *     concurrently;
 *   - matrices are row-major double[16] (MatrixTransformation::matrix,
 *     transformation.rs:47-51); an rt_transformation carries the matrix AND the
 *     separately-built inverse, exactly like the reference (the rotation "inverse"
 *     is Rx(-x)Ry(-y)Rz(-z), not a true inverse: transformation.rs:149-159).
 */
#ifndef RT_ABI_H
#define RT_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 1

typedef enum rt_status {
  RT_OK = 0,
  RT_ERR_INVALID = -1,      /* bad argument / handle / range                         */
  RT_ERR_PARSE = -2,        /* scene text does not parse (scene_loader.rs:35)         */
  RT_ERR_EVAL = -3,         /* scene evaluation error (the reference panics)          */
  RT_ERR_IO = -4,           /* texture file missing / undecodable                     */
  RT_ERR_DEVICE = -5,       /* HIP error, no GPU, or kernel launch failure            */
  RT_ERR_UNSUPPORTED = -6,  /* outside this build's limits (e.g. max_depth > 16)      */
  RT_ERR_NOMEM = -7,
  RT_PENDING = 1            /* not an error: still in progress (rt_ctx_spec_wait's time limit) */
} rt_status;

typedef enum rt_csg_op { RT_CSG_UNION = 0, RT_CSG_INTERSECTION = 1, RT_CSG_DIFFERENCE = 2 } rt_csg_op;

typedef struct rt_transformation {   /* MatrixTransformation (transformation.rs:47-51) */
  double matrix[16];
  double inverse[16];
} rt_transformation;

typedef struct rt_material {         /* SolidColorMaterial / TexturedMaterial (material.rs:34-102) */
  double color[4];                   /* r,g,b,a; ignored when texture >= 0                      */
  int32_t texture;                   /* texture id from rt_scene_add_texture, or -1 (solid)     */
  double reflectivity;
  double transparency;
} rt_material;

typedef struct rt_ray_record {       /* one RayDebuggerCallback call (raytracer.rs:17-19) as RayInfo */
  int32_t depth;
  int32_t ray_type;                  /* RayType: 0 NormalRay, 1 ReflectionRay, 2 TransmissionRay */
  int32_t object;                    /* intersected object, draw index; -1 = none */
  int32_t intersected;               /* distance != INFINITY (ray_debugger.rs:105) */
  int32_t has_normal;
  int32_t pad;
  double point[3], direction[3];     /* the ray */
  double distance;                   /* INFINITY on a miss */
  double intersection[3];            /* point + direction * (distance, or 1000 on a miss) */
  double normal[3];                  /* object shape's get_normal at the intersection (not normalised) */
  double color[4];                   /* the colour get_ray_color returns for this ray */
} rt_ray_record;

typedef struct rt_scene rt_scene;    /* a RayTracer (raytracer.rs:21-35): objects, lights, camera */
typedef struct rt_ctx rt_ctx;        /* per-device context: device scene, scratch, timing events */

/* ---- library ---------------------------------------------------------------------------- */
int rt_abi_version(void);
const char* rt_last_error(void);

/* ---- transformations (replace MatrixTransformation constructors, transformation.rs:104-205) */
int rt_xform_identity(rt_transformation* out);                                   /* :104-113 */
int rt_xform_translation(double x, double y, double z, rt_transformation* out);  /* :164-180 */
int rt_xform_rotation(double x, double y, double z, rt_transformation* out);     /* :115-162 */
int rt_xform_scaling(double x, double y, double z, rt_transformation* out);      /* :182-198 */
/* self.compose_with(other): matrix = other.m * self.m, inverse = self.inv * other.inv (:200-205);
 * TransformationStack::push_transformation(t) == compose(t, top) (:21-28). */
int rt_xform_compose(const rt_transformation* self_, const rt_transformation* other,
                     rt_transformation* out);

/* ---- scene construction (the RayTracer the scene parser fills) ------------------------- */
/* RayTracer::new_default(width, height): camera at (0,0,-100), max_depth 10 (raytracer.rs:38-70) */
int rt_scene_new(uint32_t width, uint32_t height, rt_scene** out);
/* RayTracer::add_test_objects: the always-present light (-10,30,-50) rgb .5 (raytracer.rs:125-129) */
int rt_scene_add_test_objects(rt_scene* scene);
/* Textures: RGBA8 row-major, as lodepng::decode32_file returns them (sceneparser/texture.rs:20-40).
 * The pixels are copied.  Returns the texture id (>= 0) or a negative rt_status. */
int rt_scene_add_texture(rt_scene* scene, uint32_t width, uint32_t height, const uint8_t* rgba8);
/* Shapes (math_shapes.rs / csg.rs constructors as reached from Shape::to_rt_object,
 * sceneparser/shape.rs:42-93).  Each returns a shape id (>= 0) or a negative rt_status.
 * Shapes are immutable values; one id may be used in several objects / CSG nodes. */
int rt_shape_sphere(rt_scene* scene, const rt_transformation* t, const double center[3], double radius); /* :28-39 */
int rt_shape_cube(rt_scene* scene, const rt_transformation* t, const double center[3], double length);   /* :227-245 */
int rt_shape_plane(rt_scene* scene, const rt_transformation* t, const double normal[3], double distance);/* :154-156 */
/* CSG::new(a, b, op) (csg.rs:15-31).  The children's own RTObject materials never reach the
 * shading (only the top-level object's material is read, raytracer.rs:170,190,237-238), so
 * none is taken here. */
int rt_shape_csg(rt_scene* scene, rt_csg_op op, int32_t a, int32_t b);
/* RayTracer::add_object(RTObject::new(shape, material)) (raytracer.rs:309-311, rt_object.rs:13-20) */
int rt_scene_add_object(rt_scene* scene, int32_t shape, const rt_material* material);
/* RayTracer::add_light(PointLight::new(point, color, fade_distance)) (raytracer.rs:305-307) */
int rt_scene_add_light(rt_scene* scene, const double point[3], const double color[4], double fade_distance);
/* PerspectiveCamera::new(width, height, center, None, None, None) with the centre ALREADY in
 * world space (raytracer.rs:289-299 applies the transform; the DSL applies it once before). */
int rt_scene_set_camera(rt_scene* scene, const double center[3]);
int rt_scene_set_max_depth(rt_scene* scene, int32_t max_depth);                  /* raytracer.rs:65 */
/* Whole-scene front end: restates load_scene (scene_loader.rs:24-47) on a fresh
 * new_default()+add_test_objects() RayTracer (debug_window.rs:53-62), with the global `time`
 * set (time = frame / 300 in the reference GUI).  Texture paths resolve against asset_dir
 * (NULL = CWD).  On RT_ERR_PARSE *out still receives the default scene (the reference prints
 * the error and renders the empty scene, debug_window.rs:58-60); on other errors *out = NULL. */
int rt_scene_compile(const char* scene_text, const char* asset_dir, double time,
                     uint32_t width, uint32_t height, rt_scene** out);
int rt_scene_info(const rt_scene* scene, int32_t* n_objects, int32_t* n_lights, int32_t* n_leaves,
                  uint32_t* width, uint32_t* height);
/* Introspection (tests, debuggers): the camera as PerspectiveCamera::new builds it
 * (camera.rs:30-54): out = center[3], direction[3], right[3], up[3], aspect_ratio. */
int rt_scene_get_camera(const rt_scene* scene, double out[13]);
/* The device traversal order (tests): the object hierarchy the kernels walk, as n nodes in
 * pre-order, node i = (obj[i], skip[i]); obj = -1 for a group node, skip = index after the
 * node's subtree.  Object nodes appear in draw order.  Writes min(n, cap) nodes; *n = total. */
int rt_scene_traversal(const rt_scene* scene, int32_t* obj, int32_t* skip, int32_t cap, int32_t* n);
/* The flattened scene as text (tests, debugging; no reference counterpart): the kernel-choice
 * flags, both object hierarchies and every object's and leaf's culling record -- what
 * rt_ctx_upload would put in HBM.  Writes at most cap - 1 bytes and a NUL; *len = full length. */
int rt_scene_describe(const rt_scene* scene, char* buf, size_t cap, size_t* len);
/* Light i: point[3] (world space, as stored by add_light) and color[4]. */
int rt_scene_get_light(const rt_scene* scene, int32_t i, double point[3], double color[4]);
void rt_scene_free(rt_scene* scene);

/* ---- device rendering (replaces RayTracer::get_pixel + DebugWindow::render_lines) ------ */
int rt_device_count(int* count);
int rt_ctx_create(int device, rt_ctx** out);
/* Flatten the scene to its HBM layout and copy it (and its textures) to the device, once per
 * scene.  The scene may be freed afterwards. */
int rt_ctx_upload(rt_ctx* ctx, const rt_scene* scene);
/* Render full-frame rows [y0, y1) -- the camera always uses the full (W, H), so tiles compose
 * (debug_window.rs:74-87 with `line_range` = y0..y1, pixel (x, y) -> get_pixel(x as f64, y as
 * f64)).  Output RGBA8, row (y - y0) at rgba8 + (y - y0) * row_stride_bytes; each channel is
 * `(c * 255.0) as u8` (easy_pixbuf.rs:49-52), R,G,B,A order.  rgba8 may be a device pointer
 * (written by the kernel on `stream`, asynchronously) or a host pointer (rendered into the
 * context's scratch and copied back; synchronous).  max_depth < 0 uses the scene's.
 * Tile order: the first launch of a row geometry (rows, bands, depth, f64) of >= 2048 8x8 tiles
 * on a context also records every tile's time and returns only after the host has sorted the
 * tiles (synchronous, once per geometry; an rt_ctx_upload drops the orders unless the new scene
 * has the previous one's structure -- the same scene rebuilt, an animation's next frame -- so a
 * host that re-uploads every frame keeps them); later launches of that geometry
 * dispatch the costliest tiles first.  A context keeps the orders of its 8 most recently used
 * geometries; an order table is written once and never rewritten while launches on any stream
 * may read it.  Smaller launches are dispatched row-major.  The pixels are identical either
 * way.  RT_TILE_ORDER=0 in the environment disables it. */
int rt_render_rows(rt_ctx* ctx, uint32_t y0, uint32_t y1, int32_t max_depth,
                   uint8_t* rgba8, size_t row_stride_bytes, void* stream);
/* Band layout for multi-GPU row tiling: n_bands bands of band_rows rows, band b covering
 * full-frame rows [y_first + b*band_pitch, ... + band_rows) (rows >= H skipped), written
 * packed: band b row j at output row b*band_rows + j.  A contiguous tile is n_bands = 1; the
 * cyclic layout of rank r of G uses y_first = r*band_rows, band_pitch = G*band_rows. */
int rt_render_row_bands(rt_ctx* ctx, uint32_t y_first, uint32_t band_rows, uint32_t band_pitch,
                        uint32_t n_bands, int32_t max_depth, uint8_t* rgba8, size_t row_stride_bytes,
                        void* stream);
/* Frame assembly after the multi-GPU all-gather (the GTK thread's apply_line placing every
 * worker's rows at their y, debug_window.rs:147-163, for all ranks at once).  `gathered` holds
 * `world` slots of slot_rows rows in rank order, each rank's rt_render_row_bands output for the
 * band layout above: frame row y is in band b = y / band_rows, which rank b % world packed at its
 * slot row (b / world) * band_rows + y % band_rows (a contiguous tile per rank: band_rows =
 * slot_rows).  Writes frame rows [0, height) of row_bytes bytes.  Device pointers only, one launch
 * on `stream`, asynchronous. */
int rt_assemble_row_bands(const uint8_t* gathered, size_t gathered_stride, uint32_t world, uint32_t slot_rows,
                          uint32_t band_rows, uint32_t height, size_t row_bytes, uint8_t* frame,
                          size_t frame_stride, void* stream);
/* The band layout above written as packed RGB8 (3 bytes per pixel, R,G,B; alpha is always 255):
 * the multi-GPU all-gather then moves 3/4 of the bytes.  row_stride_bytes >= 3 * width. */
int rt_render_row_bands_rgb8(rt_ctx* ctx, uint32_t y_first, uint32_t band_rows, uint32_t band_pitch,
                             uint32_t n_bands, int32_t max_depth, uint8_t* rgb8, size_t row_stride_bytes,
                             void* stream);
/* rt_assemble_row_bands from gathered packed RGB8 slot rows (rt_render_row_bands_rgb8) into RGBA8
 * frame rows (A = 255, the bytes rt_render_rows writes): `width` pixels per row; frame rows 4-byte
 * aligned.  Device pointers only, one launch on `stream`, asynchronous. */
int rt_assemble_row_bands_rgb8(const uint8_t* gathered, size_t gathered_stride, uint32_t world, uint32_t slot_rows,
                               uint32_t band_rows, uint32_t height, uint32_t width, uint8_t* frame,
                               size_t frame_stride, void* stream);
/* Same as rt_render_rows, pre-quantisation colours: 4 doubles per pixel (r,g,b,a) -- the
 * `Vec<Color>` rows. */
int rt_render_rows_f64(rt_ctx* ctx, uint32_t y0, uint32_t y1, int32_t max_depth,
                       double* rgba_f64, size_t row_stride_bytes, void* stream);
/* Arbitrary sample positions (the anti-aliaser's fractional get_pixel calls,
 * antialiaser.rs:108-112): xy = n pairs of doubles, out = n x 4 doubles. Device or host. */
int rt_render_points_f64(rt_ctx* ctx, const double* xy, size_t n, int32_t max_depth,
                         double* rgba_f64, void* stream);
/* One sample of a scene without a context of the caller's: RayTracer::get_pixel(x, y)
 * (raytracer.rs:359-365) as SURVEY 8(b) sketches it for hosts that trace single pixels (a debugger
 * UI, an anti-aliaser driven pixel by pixel).  Traced on the GPU (`device`, a context of the calling
 * thread kept for the next call; the scene is uploaded on every call, so an edited scene is seen):
 * about a millisecond per call -- batches belong in rt_render_points_f64.  max_depth < 0: the
 * scene's.  rgba = 4 doubles, host memory. */
int rt_trace_pixel_f64(const rt_scene* scene, double x, double y, int32_t max_depth, int device, double rgba[4]);
/* Ray-debugger recording (RayDebugger::record_rays, ray_debugger.rs:92-137): trace pixel (x, y)
 * (fractional allowed) once with the debugger callback attached and return one record per ray in
 * the reference's callback order (a ray reports after its children).  *n_rays = rays traced
 * (records past cap are dropped); rgba (may be NULL) = get_pixel's colour.  Host pointers;
 * synchronous.  Not a throughput path. */
int rt_record_rays(rt_ctx* ctx, double x, double y, int32_t max_depth, rt_ray_record* records, int32_t cap,
                   int32_t* n_rays, double* rgba);
/* Orthogonal preview view (DebugWindow::render_orthogonal_view_line, debug_window.rs:166-227)
 * for rows [y0, y1) at the scene's W x H: per pixel a ray from 10000 along the third axis with
 * origin[axis1] = ((x - W/2) * dir1) / scale, origin[axis2] = ((y - H/2) * dir2) / scale; the
 * object with the smallest intersection distance (any sign, no EPS) gives its flat colour
 * (RTObject::get_color, rt_object.rs:45-47), a miss is (0,0,0,0).  The GUI's views are
 * OrthoAxes (ray_debugger.rs:33-68): top (0,2,+1,-1,2), front (0,1,+1,-1,2), side (2,1,-1,-1,2).
 * Either output may be NULL (not both); device or host pointers.  RT_ERR_INVALID for invalid
 * axes (the reference panics). */
int rt_render_ortho(rt_ctx* ctx, int32_t axis1, int32_t axis2, double dir1, double dir2, double scale,
                    uint32_t y0, uint32_t y1, uint8_t* rgba8, size_t row_stride_bytes, double* rgba_f64,
                    size_t f64_stride, void* stream);
/* Adaptive anti-aliasing pass (antialiaser.rs:87-191, driven as debug_window.rs:275-320) over a
 * QUANTISED frame of the uploaded scene's size: corners come from src (u8 / 255), interior
 * sub-pixels are traced at (x + i/size, y + j/size), size = 2^level + 1; a cell subdivides while
 * the mean |dRGBA| of its corners exceeds threshold and level > 0.  Writes the whole frame to
 * dst_rgba8 and/or dst_f64 (either may be NULL, not both); the last column and row are the source
 * pixels (the reference never anti-aliases them).  level <= 4.  *rays_traced (may be NULL) = the
 * reference's ray_counter.  Pointers may be device or host; the call returns when the frame is
 * done (the pass sizes its work from the edge count).  Replaces AntiAliaser::get_anti_aliased_pixel
 * over every pixel (antialiaser.rs:53-71, :87-122). */
int rt_antialias(rt_ctx* ctx, const uint8_t* src_rgba8, size_t src_stride, double threshold, int32_t level,
                 int32_t max_depth, uint8_t* dst_rgba8, size_t dst_stride, double* dst_f64, size_t f64_stride,
                 uint64_t* rays_traced, void* stream);
/* Milliseconds of the last render launch on this context (HIP events recorded on the launch's
 * stream around the kernel; RT_OPT_TIMING 0 turns them off and this call then fails). */
int rt_ctx_last_kernel_ms(rt_ctx* ctx, float* ms);
/* Waits until every launch this context made has finished, on whichever streams (each launch records
 * a completion event of the context's own; the callers' streams are never touched, so they may have
 * been destroyed). */
int rt_ctx_synchronize(rt_ctx* ctx);
/* Tuning options of a context.  No option changes a single pixel; they only choose how the
 * kernels run.  RT_OPT_KERNEL selects the render kernel for scenes without a transparent object:
 *   RT_KERNEL_AUTO (default): a launch bound by its costliest tiles (fewer tiles than ~5 per wave
 *     slot, costliest tile > the work per slot) takes the deferred-shadow kernel with the costly
 *     tiles split over several waves, every other launch the per-lane megakernel;
 *   RT_KERNEL_MEGA: always the megakernel -- best when several frames are in flight on different
 *     streams (their launches overlap, so no launch's tail leaves the GPU idle);
 *   RT_KERNEL_DEFERRED: always the deferred-shadow kernel (scenes whose rays form chains);
 *   RT_KERNEL_WAVEFRONT: the launch-wide wavefront path for any scene: one pass per recursion depth
 *     over a dense queue of that depth's rays, then a bottom-up fold (k_wavefront.hip wf_*).
 * Changing the kernel drops the context's tile orders (the next launch of each geometry
 * calibrates again).  Scenes with a transparent object always take the refraction megakernel.
 * RT_OPT_TIMING: 1 (default) records a HIP event pair around every render launch for
 * rt_ctx_last_kernel_ms; 0 records none.  Each timed event costs the stream ~5 us on MI355X
 * (a 1080p single-sphere frame: 0.045 -> 0.036 ms per launch without them), so a host that
 * times its own stream, or does not time at all, turns them off.
 * RT_OPT_TILE_ORDER: 1 (default) dispatches the tiles of a geometry longest-first after one
 * calibration launch (a host synchronisation per new geometry); 0 dispatches row-major.
 * RT_OPT_FAST_CLAMP: 1 (default) lets the kernels clamp colours with min/max where the host proved
 * it bit-identical to the reference's compare/select clamp (RtDevScene::colour_fast); 0 keeps the
 * compare/select form everywhere (A/B checks).
 * RT_OPT_WAVEFRONT_CAP: rays each recursion level of the wavefront path holds, in percent of the
 * launch's pixel slots (1..400, default 200); a pixel whose ray tree overflows a level is rendered
 * again by the per-lane megakernel (same bits), so the value trades memory against that fallback.
 * RT_OPT_WAVEFRONT_PAIRS: how the wavefront path traces a level's rays: 0 one wave walks the object
 * hierarchy for 64 rays (wf_trace_kernel); 1 (default) levels >= 1 go through (ray, object) pairs
 * sorted by object, so a wave tests one object against 64 rays (wfp_* kernels; scenes whose shadow
 * products are order-free, RtDevScene::shadow_pow, and fewer than 4096 objects; else as 0); 2 level 0
 * (the camera rays) too.  The wavefront path synchronises the host with the launch stream once per
 * launch on the pair path (its levels read their ray counts on the device; the host checks the pair
 * lists' capacity at the end) and once per recursion level on the wave walk (it reads each level's ray
 * count), and RT_KERNEL_AUTO's first ordered launch of a ray-tree geometry times one wavefront launch
 * against the megakernel (blocking, once): such launches return only after the work is done, even with
 * device output.
 * RT_OPT_SPECIALIZE: 1 (default) compiles the uploaded scene's row kernels once more with the scene's
 * tables as constants (hipRTC, spec.hip: the hierarchy walk unrolled, every record field a literal;
 * same pixels) for RGBA8 / RGB8 launches; 2 for the f64 and calibration launches too; 0 never.  The
 * compile is ASYNCHRONOUS: rt_ctx_upload (or this call) requests it from a pool of library threads
 * and returns at once; launches take the generic kernels until the code objects are ready and the
 * specialised ones from the first launch after (rt_ctx_kernel_info says which ran).  The first frame
 * therefore renders as fast as without the option, and the compile (seconds of host time on a new
 * scene; 4K globes: 0.457 -> 0.325 ms per frame once loaded) costs the host thread nothing.
 * rt_ctx_spec_wait blocks for it.  Programs are cached per process by their full text, and on disk
 * (rt_spec_cache_dir) by text, compiler, embedded device headers and compile options.  Scenes of more than 32 objects or 48 leaves keep the
 * generic kernels (the unrolled walks grow with the scene), and so does a context whose compile
 * failed or whose code object exceeds the resource guard, or when the ROCm installation's hipRTC
 * cannot be loaded (rt_ctx_kernel_info says why; the upload itself succeeds).  Setting the same
 * value again after a failure retries the compile.  Launches whose kernel has no specialised form
 * (wavefront, refraction deferred, RT_OPT_FAST_CLAMP 0 on a min/max-clamp scene) keep the generic
 * kernels.
 * Option 7 is retired (round 4's tail kernel, measured slower than the launch it shortened). */
typedef enum rt_option {
  RT_OPT_KERNEL = 0, RT_OPT_TIMING = 1, RT_OPT_TILE_ORDER = 2, RT_OPT_FAST_CLAMP = 3, RT_OPT_WAVEFRONT_CAP = 4,
  RT_OPT_WAVEFRONT_PAIRS = 5, RT_OPT_SPECIALIZE = 6
} rt_option;
typedef enum rt_kernel_choice {
  RT_KERNEL_AUTO = 0, RT_KERNEL_MEGA = 1, RT_KERNEL_DEFERRED = 2, RT_KERNEL_WAVEFRONT = 3
} rt_kernel_choice;
int rt_ctx_set_option(rt_ctx* ctx, int32_t option, int32_t value);
/* What the context's row launches run, as text: "generic (librt_mi355x.so...)" -- with the reason when
 * RT_OPT_SPECIALIZE is on (compiling in the background, failed, scene too large) -- or the specialised
 * program's hash, mode, compile time, compiler and resources, and which kernel the last row launch took. */
int rt_ctx_kernel_info(rt_ctx* ctx, char* buf, size_t cap);
/* Block until the context's specialised program (RT_OPT_SPECIALIZE) is loaded, at most timeout_ms
 * (< 0: no limit).  RT_OK: loaded, or nothing to wait for (option off, scene too large); RT_PENDING:
 * the limit passed first; a negative status: the compile failed or the guard refused it (the
 * context keeps the generic kernels, rt_last_error / rt_ctx_kernel_info say why). */
int rt_ctx_spec_wait(rt_ctx* ctx, int32_t timeout_ms);
/* Compile the scene's specialised program (RT_OPT_SPECIALIZE) into the process's code-object
 * cache without a device, so a later upload of the same scene finds it; *compile_ms = the hipRTC
 * time (0 when it was cached already).  May run on any thread. */
int rt_scene_precompile(const rt_scene* scene, double* compile_ms);
/* rt_scene_precompile, then a report of the programs as text (cap, len as rt_scene_describe): the
 * compiler's identity, and per kernel "NAME: vgprs V spilled S sgprs G scratch B occupancy W code N
 * compile_ms T source hiprtc|disk" (the code object's metadata: what the resource guard checks). */
int rt_scene_spec_report(const rt_scene* scene, char* buf, size_t cap, size_t* len);
/* The hipRTC the programs compile with (its path, version, real path, size and mtime) and "build H",
 * H = a hash of the device headers this library embeds and the compile options: together the disk-cache
 * identity.  *rocm = 1 when it is the ROCm installation's own ($ROCM_PATH or /opt/rocm), loaded into a
 * link-map namespace of its own; 0 when that failed (then nothing is specialised: the process's own
 * hipRTC may be another LLVM -- PyTorch bundles one -- whose code ran 19x slower). */
int rt_spec_compiler_info(char* buf, size_t cap, int32_t* rocm);
/* The on-disk code-object cache of the specialised programs: a directory (created on first write);
 * NULL or "" (the default) for none.  Entries are keyed by the full program text and the identity of
 * rt_spec_compiler_info (compiler, embedded headers, options); both are compared on a hit, and the
 * resources the guard checks are read from the stored code object itself. */
int rt_spec_cache_dir(const char* dir);
/* Stop the compile pool before the process exits: queued compiles are cancelled, running ones are
 * waited for (a compile still running in a library thread while the process tears hipRTC down could
 * crash the exit).  Later requests fail (contexts keep the generic kernels).  The library registers it
 * with atexit() when its first compile thread starts, so a host that never calls it is covered too;
 * calling it again is harmless. */
void rt_spec_shutdown(void);
/* The specialised program's text (tests, debugging): cap, len as rt_scene_describe. */
int rt_scene_spec_program(const rt_scene* scene, char* buf, size_t cap, size_t* len);
/* Specialised programs for n scenes -- the frames of an animation (the reference's animate mode
 * builds every frame's scene anew, gui.rs:78-89) -- one per FAMILY of scenes of the same structure:
 * equal table sizes, object hierarchy, CSG nodes, filter programs, textures and flags; the numbers
 * may differ.  The words of the flattened tables every member of a family shares are compiled in
 * as constants, the others are read from the rendering scene's own tables, so a family's one
 * hipRTC compile serves all its members (the families compile in parallel; *compile_ms = the
 * longest, 0 if all were cached).  Registered for the process: a context with RT_OPT_SPECIALIZE
 * whose uploaded scene matches a registered family (a member, or any scene sharing those words)
 * loads the family's program instead of compiling its own (newest first); set the option after
 * registering, or upload after it.  RT_ERR_UNSUPPORTED: scenes above the specialisation limits.
 * Same pixels as the generic kernels. */
int rt_spec_family_register(const rt_scene* const* scenes, int32_t n, double* compile_ms);
/* Forget every registered family (contexts keep the programs they loaded). */
int rt_spec_family_clear(void);
void rt_ctx_free(rt_ctx* ctx);
/* A HIP stream on a hardware queue of its own (hipExtStreamCreateWithCUMask with every CU
 * enabled), for renders that overlap: plain streams share the process's few hardware queues
 * (GPU_MAX_HW_QUEUES, 4 by default) and two overlapping renders whose streams land on one queue
 * run one after the other (measured: a rank's N = 8 share with 4 frames in flight 0.118 instead
 * of 0.071 ms).  The reference renders on a thread pool (gui.rs:49-51); streams are its
 * MI355X counterpart.  *stream is a hipStream_t; free it with rt_stream_destroy. */
int rt_stream_create(int device, void** stream);
int rt_stream_destroy(void* stream);

/* ---- output ----------------------------------------------------------------------------- */
/* PNG encoder for the headless driver (the reference has none; it only paints a cairo
 * surface).  channels = 3 (RGB, alpha dropped) or 4. Host pointer. */
int rt_write_png(const char* path, const uint8_t* rgba8, uint32_t width, uint32_t height,
                 size_t row_stride_bytes, int channels);
/* PNG decoder used for textures (lodepng::decode32_file equivalent). *pixels is malloc'd;
 * release with rt_free_buffer. */
int rt_read_png_rgba8(const char* path, uint8_t** pixels, uint32_t* width, uint32_t* height);
void rt_free_buffer(void* p);

#ifdef __cplusplus
}
#endif
#endif /* RT_ABI_H */
