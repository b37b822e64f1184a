/*
 * rt_scene.h — host-side scene ingest of the path-tracer hot path (C-ABI, exported by
 * librt_hip.so; pure host code, no device needed).
 *
 * Replaces the reference's Swift scene layer feeding raytracingKernel:
 *   Scene.init / lights / camera        MetalRaytracing/Scene.swift:73-169
 *   AppScene model list                 MetalRaytracing/AppScene.swift:11-28
 *   Model.init (OBJ path), transforms   MetalRaytracing/Model.swift:45-196, Utilities.swift:302-355
 *   Mesh / Submesh buffers, materials   MetalRaytracing/Mesh.swift:17-68, SubMesh.swift:56-324
 *   Renderer.updateUniforms defaults    MetalRaytracing/Renderer.swift:116-192, :608-664
 *   random-offset texture               MetalRaytracing/Renderer.swift:709-738
 * The description it produces (rt_scene_desc, rt_api.h) is what rt_scene_upload consumes.
 */
#ifndef RT_SCENE_H
#define RT_SCENE_H

#include "rt_types.h"
#include "rt_api.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rt_scene rt_scene;

/* ModelMaterialOverride (Model.swift:11-27). A field is applied when its has_* flag is set. */
typedef struct rt_material_override {
    int32_t has_base_color;
    float base_color[3];
    int32_t has_refraction_index;
    float refraction_index;
    int32_t has_opacity;
    float opacity;
} rt_material_override;

/* ModelMaterialOverride.glass() defaults: tint (0.95,0.98,1.0), ior 1.52, opacity 0.08. */
void rt_material_override_glass(rt_material_override* out);

/* Empty scene with the reference's default lights (area light + spotlight, Scene.swift:82-91). */
rt_status rt_scene_new(rt_scene** out);
rt_status rt_scene_free(rt_scene* scene);
const char* rt_scene_last_error(const rt_scene* scene);

/* Model(name:position:rotation:scale:materialOverride:) for an OBJ asset (Model.swift:45-196).
 * `obj_path` is a path to a .obj file; its mtllib is resolved relative to the .obj. Fails with
 * RT_ERR_IO when the file is missing (the reference fatalErrors, Model.swift:68-70). */
rt_status rt_scene_add_obj(rt_scene* scene, const char* obj_path, const float position[3],
                           const float rotation[3], float scale, const rt_material_override* ov);

/* Model(name:position:rotation:scale:materialOverride:) for a USD asset — the USDZ branch of
 * Model.init (Model.swift:87-184).  `usd_path` is a .usdz package (its first .usd/.usda/.usdc
 * entry is the root layer; textures are read from the package), a .usda text layer or a .usdc
 * crate layer.  Every active UsdGeomMesh becomes one mesh in depth-first order, placed by the
 * model's T*R*S only (the reference passes worldTransform to every mesh, Model.swift:162-170):
 * fan-triangulated faces, one vertex per unique (point, normal, uv) corner, normals computed
 * when absent, one submesh per materialBind GeomSubset, UsdPreviewSurface inputs mapped as
 * Material(material:) does (SubMesh.swift:291-324) plus their texture maps.  The last Skeleton
 * and SkelAnimation met in the walk are the model's (Model.swift:99-121); meshes carrying
 * skel:jointIndices / jointWeights become skinned meshes (first four influences), their joint
 * order (skel:joints or the skeleton's) mapped to the skeleton by path, unique suffix and tail
 * (Model.swift:427-494).  Composition arcs (references, payloads, variants) are not followed.
 * Fails with RT_ERR_IO when the file is missing or malformed. */
rt_status rt_scene_add_usd(rt_scene* scene, const char* usd_path, const float position[3], const float rotation[3],
                           float scale, const rt_material_override* ov);

/* Deterministic procedural stand-ins for the assets missing from the reference snapshot
 * (.MISSING_LARGE_BLOBS): kind = "dragon" (871,414 tris), "bunny" (69,451 tris),
 * "robot" (skinned, for config 5). `mtl_path` may be NULL (built-in material). */
rt_status rt_scene_add_procedural(rt_scene* scene, const char* kind, const char* mtl_path,
                                  const float position[3], const float rotation[3], float scale,
                                  const rt_material_override* ov);

/* Replace the light list (Scene.lights). */
rt_status rt_scene_set_lights(rt_scene* scene, const Light* lights, uint32_t count);
/* Scene.setLightIntensity (Scene.swift:57-63). */
rt_status rt_scene_set_light_intensity(rt_scene* scene, float intensity);

/* Benchmark / parity presets: "c1", "c2", "c3", "c3g", "c3d", "c5", "app"; "c3r" (the
 * reference's coatball / teapot meshes in the dragon's place, glass: an irregular-geometry check). 
 * `asset_dir` holds the OBJ/MTL files (plane.obj, sphere.obj, ...); a real dragon.obj /
 * bunny.obj / robot.usdz found there is loaded instead of the procedural stand-in unless the
 * preset name ends in "_synthetic". *is_synthetic reports whether a stand-in was used. */
rt_status rt_scene_preset(const char* name, const char* asset_dir, rt_scene** out, int32_t* is_synthetic);

/* Flattened description. Pointers stay valid until the scene is modified or freed. */
rt_status rt_scene_get_desc(rt_scene* scene, rt_scene_desc* out);

/* Textures (SubMesh.swift:69-241).  add_texture copies width x height RGBA8 texels (row 0 = top);
 * load_texture decodes a PNG file (the MTKTextureLoader stand-in).  bind_texture attaches texture
 * `texture_id` to slot `slot` (RT_TEXTURE_SLOTS order) of submesh `submesh_index` of the scene's
 * mesh `mesh_index` (the flattened mesh order of rt_scene_get_desc), sets the slot's
 * textureFlags bit and, for the base color slot, baseColor = 1 (SubMesh.swift:120-124).
 * OBJ materials bind their MTL maps when the files decode: map_Kd (base color), norm / bump /
 * map_Bump (normal), map_Pr (roughness), map_Pm (metallic), map_Ke (emission), map_d
 * (opacity); a map that fails to load leaves its slot unbound, as the reference's loader does. */
rt_status rt_scene_add_texture(rt_scene* scene, const uint8_t* rgba8, uint32_t width, uint32_t height, uint32_t* id);
rt_status rt_scene_load_texture(rt_scene* scene, const char* png_path, uint32_t* id);
rt_status rt_scene_bind_texture(rt_scene* scene, uint32_t mesh_index, uint32_t submesh_index, uint32_t slot,
                                uint32_t texture_id);

/* PNG decode into RGBA8 (row 0 = top): call with rgba8 = NULL for the size, then with a buffer
 * of width * height * 4 bytes.  err_buf (optional) receives the reason of a failure. */
rt_status rt_decode_png(const uint8_t* data, size_t size, uint8_t* rgba8, uint32_t* width, uint32_t* height,
                        char* err_buf, size_t err_len);
/* Writes width x height RGBA8 rows (row 0 = top) as an 8-bit RGBA PNG (e.g. rt_present output). */
rt_status rt_write_png(const char* path, const uint8_t* rgba8, uint32_t width, uint32_t height);
/* Totals for reports. */
uint64_t rt_scene_triangle_count(const rt_scene* scene);

/* Skinned meshes (config 5): joint matrices for animation time t, already composed as
 * geomBind^-1 * (global * invBind) * geomBind (SkinningPass.swift:124-157, Model.swift:207-261).
 * For a USD model: Model.update's clip time fmod(t, duration), the animation's translations /
 * rotations / scales sampled there (linear, rotations spherical; clamped outside the keys; time
 * codes / timeCodesPerSecond), local = T * R(normalised q) * S over the rest transforms,
 * global = parent global * local, skin = global * inverse bind, one matrix per mesh joint
 * (identity for joints the skeleton lacks).  `out` receives joint_count column-major float4x4. */
rt_status rt_scene_joint_matrices(rt_scene* scene, uint32_t mesh_index, double time_seconds,
                                  float* out, uint32_t capacity, uint32_t* joint_count);

/* Scene.setupCamera / makeOrbitCamera (Scene.swift:111-159). */
void rt_camera_default(int32_t width, int32_t height, Camera* out);
void rt_camera_orbit(int32_t width, int32_t height, const float target[3], float azimuth,
                     float elevation, float distance, float fov_degrees, Camera* out);

/* Renderer knob defaults written by updateUniforms (Renderer.swift:116-192, :608-664):
 * spp 2, maxBounces 2, accumulationWeight 0.9, motion-adaptive accumulation on (0.1, 0.5-4 px),
 * motion-adaptive sampling on (+2, 1-6 px), PBR, debug 0, G-buffer off, frameIndex 0,
 * camera = previousCamera = default orbit camera, lightCount as given. */
void rt_uniforms_default(int32_t width, int32_t height, int32_t light_count, Uniforms* out);

/* Per-pixel decorrelation offsets: splitmix64(seed) % 2^20 in row-major order — the seeded
 * substitute for arc4random() % (1024*1024) (Renderer.swift:719-738). */
void rt_random_offsets(uint64_t seed, int32_t width, int32_t height, uint32_t* out);

#ifdef __cplusplus
}
#endif
#endif /* RT_SCENE_H */
