/* pt_scene.h -- host-side scene ingest for the MI355X path tracer (C ABI, no GPU needed).
 *
 * Replaces the reference's host scene pipeline, which feeds the compute shader's SSBOs:
 *   load_vertex_data()   LearnOpenGL/header_files/geometry_loader.h:15-142  -> pt_scene_load_obj
 *   buildSAHTree()       LearnOpenGL/header_files/bvh.h:255-268             -> pt_scene_build_bvh / pt_bvh_build
 *   setupBuffers()       LearnOpenGL/header_files/ogl_path_trace.h:367-530  -> pt_scene_add_builtins
 *
 * All arrays use the reference's std140 AoS records (computeShader.c:7-35), float4-packed:
 *   triangle  16 floats  {v0.xyzw, v1.xyzw, v2.xyzw, {matIdx, 0, 0, 0}}       (triangle.h:8-15)
 *   material  16 floats  {color, emissionColor, specularColor,
 *                         {emissionStrength, smoothness, specularProbability, 0}} (material.h:5-12)
 *   sphere     8 floats  {{c.xyz, r}, {matIdx, 0, 0, 0}}                         (sphere.h:7-11)
 *   bvh node  12 floats  {min.xyzw, max.xyzw, {tri0, tri1, hitLink, missLink}}   (bvh.h:15-19)
 * so the output of these calls can be handed to pt_upload_scene() (pt_api.h) unchanged.
 *
 * Errors: functions return 0 on success or a negative PT_E* code (pt_api.h); a message is
 * available from pt_scene_last_error().  Not thread-safe per scene object.
 */
#ifndef PT_SCENE_H
#define PT_SCENE_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pt_scene pt_scene;

/* Reads MTL first (exactly 8 property lines after each `newmtl`), then OBJ (`v`, `f a b c`
 * with global 1-based indices, `usemtl`); geometry_loader.h:15-142, quirks in DESIGN.md §2.3.
 * Emission strength is forced to 7.5 for loaded materials (geometry_loader.h:84). */
int pt_scene_load_obj(const char* obj_path, const char* mtl_path, pt_scene** out);

/* Loader selection for pt_scene_load_obj_ex. */
#define PT_LOAD_REFERENCE 0  /* exactly pt_scene_load_obj (the reference's parser semantics) */
#define PT_LOAD_ROBUST 1     /* general Wavefront reader: f corners v, v/vt,
                                v/vt/vn, v//vn, negative indices, polygons (fan-triangulated),
                                comments, continuations, any line length, MTL properties in any
                                order, `mtllib` when mtl_path is NULL; malformed input is a
                                PT_E_PARSE with file:line.  Same material mapping as the
                                reference (Kd, Ke, Ks, Ns/1000, strength 7.5), and the same
                                arrays on files the reference reads correctly. */
int pt_scene_load_obj_ex(const char* obj_path, const char* mtl_path, int flags, pt_scene** out);

/* Wraps caller arrays (copied) in a scene object: n_tris*16 and n_mats*16 floats. */
int pt_scene_from_arrays(const float* tris, int n_tris, const float* mats, int n_mats,
                         pt_scene** out);

/* Appends the reference's five built-in materials (light, spec, diffuse, ground, metal)
 * after the loaded ones and the one metal sphere (-0.5, 3, 1, r 0.8, material m+4):
 * ogl_path_trace.h:415-453, 498-501.  Idempotent. */
int pt_scene_add_builtins(pt_scene* s);

/* buildSAHTree: binary SAH BVH (<=2 tris per leaf, 60-candidate sweep per axis, stable
 * centroid sort) + hit/miss link threading.  Topology identical to bvh.h:173-268. */
int pt_scene_build_bvh(pt_scene* s);

/* counts: n_tris, n_mats (incl. built-ins), n_spheres, n_nodes, n_loaded_mats */
int pt_scene_counts(const pt_scene* s, int counts[5]);

/* Copy-out of the std140 buffers; each `max_*` is the capacity in records. */
int pt_scene_get_tris(const pt_scene* s, float* dst, int max_tris);
int pt_scene_get_mats(const pt_scene* s, float* dst, int max_mats);
int pt_scene_get_spheres(const pt_scene* s, float* dst, int max_spheres);
int pt_scene_get_nodes(const pt_scene* s, float* dst, int max_nodes);

const char* pt_scene_last_error(const pt_scene* s);
void pt_scene_free(pt_scene* s);

/* Stand-alone builder on raw arrays: nodes_out needs capacity >= 2*n_tris-1 nodes. */
int pt_bvh_build(const float* tris, int n_tris, float* nodes_out, int max_nodes, int* n_nodes);

/* The same builder on GPU `device`: one tree level at a time, the
 * chained stable centroid sorts as segmented device sorts, the prefix / suffix candidate
 * boxes as segmented scans, the split choice one thread per node.  Output identical to
 * pt_bvh_build (same node numbering, bounds, leaf indices and links).  Needs a GPU. */
int pt_bvh_build_gpu(const float* tris, int n_tris, float* nodes_out, int max_nodes, int* n_nodes,
                     int device);
/* pt_scene_build_bvh with the GPU builder. */
int pt_scene_build_bvh_gpu(pt_scene* s, int device);
/* 1 when the threaded tree qualifies for the culling walk: from node 0 a
 * full binary tree threaded in preorder (hit link = left child, the left child's miss link =
 * the right child, the right child's miss link = the parent's) whose internal boxes contain
 * both children's boxes exactly; else 0.  Host only; pt_upload_scene applies the same check. */
int pt_bvh_culling_ok(const float* nodes, int n_nodes);
/* Message of the calling thread's last pt_bvh_build / pt_bvh_build_gpu failure. */
const char* pt_bvh_last_error(void);

/* ACES film tonemap (screenQuadFrag.c:12-33) of an RGBA32F image to RGBA8 on the host;
 * the device form is pt_read_rgba8_aces() in pt_api.h. */
void pt_aces_rgba8_host(const float* rgba, long long n_pixels, unsigned char* out);

#ifdef __cplusplus
}
#endif
#endif /* PT_SCENE_H */
