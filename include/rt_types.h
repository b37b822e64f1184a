/*
 * rt_types.h — host/GPU shared data layout of the path-tracer hot path.
 *
 * C mirror of the reference's shared header MetalRaytracing/ShaderTypes.h:1-170
 * (tatsuya-ogawa/metal4-raytracing). Field order, sizes and offsets are identical to the
 * Metal/simd layout (vector_float3 = 16-byte size and alignment), so a buffer written by the
 * reference's Swift side (Scene.lightBuffer, the Uniforms ring, Submesh.materialBuffer) can be
 * handed to this library unchanged.  Every offset is pinned by a static assertion below
 * (SURVEY.md Appendix A).
 *
 * Plain C99/C++ — no HIP, no torch types — so it is usable from the C-ABI, the CPU oracle and
 * the HIP kernels alike.
 */
#ifndef RT_TYPES_H
#define RT_TYPES_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* simd vector_float3: 12 bytes of payload padded to 16, 16-byte aligned (ShaderTypes.h:15). */
typedef struct __attribute__((aligned(16))) rt_float3 {
    float x, y, z, _pad;
} rt_float3;

typedef struct __attribute__((aligned(8))) rt_float2 {
    float x, y;
} rt_float2;

/* ---- enums (ShaderTypes.h:35-78, :87-93, :132-135, :159-168) ---------------------------- */
enum {
    BufferIndexUniforms = 0,
    BufferIndexInstanceAccelerationStructure = 1,
    BufferIndexRandom = 2,
    BufferIndexVertexColor = 3,
    BufferIndexVertexNormals = 4,
    BufferIndexResources = 5,
    BufferIndexLights = 6,
    BufferIndexInstances = 7,
    BufferIndexAccelerationStructure = 8,
    BufferIndexInstanceDescriptors = 9,
    BufferIndexRestPositions = 10,
    BufferIndexRestNormals = 11,
    BufferIndexJointIndices = 12,
    BufferIndexJointWeights = 13,
    BufferIndexJointMatrices = 14,
    BufferIndexSkinnedPositions = 15,
    BufferIndexSkinnedNormals = 16,
    BufferIndexPreviousInstanceDescriptors = 17
};

enum {
    TextureIndexAccumulation = 0,
    TextureIndexPreviousAccumulation = 1,
    TextureIndexRandom = 2,
    TextureIndexDepth = 3,
    TextureIndexMotion = 4,
    TextureIndexDiffuseAlbedo = 5,
    TextureIndexSpecularAlbedo = 6,
    TextureIndexNormal = 7,
    TextureIndexRoughness = 8
};

enum {
    LightTypeUnused = 0,
    LightTypeSunlight = 1,
    LightTypeSpotlight = 2,
    LightTypePointlight = 3,
    LightTypeAreaLight = 4
};

enum { ShadingModePBR = 0, ShadingModeLegacy = 1 };

enum {
    DebugTextureModeNone = 0,
    DebugTextureModeBaseColor = 1,
    DebugTextureModeNormal = 2,
    DebugTextureModeRoughness = 3,
    DebugTextureModeMetallic = 4,
    DebugTextureModeAO = 5,
    DebugTextureModeEmission = 6,
    DebugTextureModeMotion = 7
};

#define MATERIAL_TEXTURE_BASECOLOR (1u << 0)
#define MATERIAL_TEXTURE_NORMAL    (1u << 1)
#define MATERIAL_TEXTURE_ROUGHNESS (1u << 2)
#define MATERIAL_TEXTURE_METALLIC  (1u << 3)
#define MATERIAL_TEXTURE_AO        (1u << 4)
#define MATERIAL_TEXTURE_EMISSION  (1u << 5)
#define MATERIAL_TEXTURE_OPACITY   (1u << 6)

#ifndef ENABLE_AO
#define ENABLE_AO 0 /* ShaderTypes.h:155-157 */
#endif

/* ---- structs ---------------------------------------------------------------------------- */

/* ShaderTypes.h:80-85. right/up are pre-scaled by the image-plane size (Scene.swift:149-157). */
typedef struct Camera {
    rt_float3 position;
    rt_float3 right;
    rt_float3 up;
    rt_float3 forward;
} Camera;

/* ShaderTypes.h:95-106. `type` is a 32-bit NSInteger on the GPU (ShaderTypes.h:21). */
typedef struct Light {
    int32_t type;
    rt_float3 position;
    rt_float3 color;
    rt_float3 forward;   /* area light */
    rt_float3 right;
    rt_float3 up;
    float coneAngle;     /* spot light (radians) */
    rt_float3 direction;
} Light;

/* ShaderTypes.h:108-130 */
typedef struct Uniforms {
    int32_t width;
    int32_t height;
    int32_t blocksWide;
    uint32_t frameIndex;
    int32_t lightCount;
    int32_t samplesPerPixel;
    int32_t maxBounces;
    Camera camera;
    Camera previousCamera;
    int32_t debugTextureMode;
    float accumulationWeight;
    int32_t enableDenoiseGBuffer;
    int32_t shadingMode;
    int32_t enableMotionAdaptiveAccumulation;
    float motionAccumulationMinWeight;
    float motionAccumulationLowThresholdPixels;
    float motionAccumulationHighThresholdPixels;
    int32_t enableMotionAdaptiveSampling;
    int32_t motionSamplingMaxExtraSamples;
    float motionSamplingLowThresholdPixels;
    float motionSamplingHighThresholdPixels;
} Uniforms;

/* ShaderTypes.h:137-145 */
typedef struct Material {
    rt_float3 baseColor;
    rt_float3 specular;
    rt_float3 emission;
    float specularExponent;
    float refractionIndex;
    float opacity;
    uint32_t textureFlags;
} Material;

/* MTLPackedFloat4x3: 4 columns of packed float3, column-major object->world
 * (Renderer.swift:1393-1401; consumed at Raytracing.metal:329-333). 48 bytes. */
typedef struct rt_packed_float4x3 {
    float columns[4][3];
} rt_packed_float4x3;

/* ---- layout pins -------------------------------------------------- */
#ifdef __cplusplus
#define RT_STATIC_ASSERT(c, m) static_assert(c, m)
#else
#define RT_STATIC_ASSERT(c, m) _Static_assert(c, m)
#endif
RT_STATIC_ASSERT(sizeof(rt_float3) == 16, "float3 is 16 B");
RT_STATIC_ASSERT(sizeof(Camera) == 64, "Camera 64 B");
RT_STATIC_ASSERT(sizeof(Light) == 128, "Light 128 B");
RT_STATIC_ASSERT(offsetof(Light, position) == 16, "Light.position@16");
RT_STATIC_ASSERT(offsetof(Light, color) == 32, "Light.color@32");
RT_STATIC_ASSERT(offsetof(Light, forward) == 48, "Light.forward@48");
RT_STATIC_ASSERT(offsetof(Light, right) == 64, "Light.right@64");
RT_STATIC_ASSERT(offsetof(Light, up) == 80, "Light.up@80");
RT_STATIC_ASSERT(offsetof(Light, coneAngle) == 96, "Light.coneAngle@96");
RT_STATIC_ASSERT(offsetof(Light, direction) == 112, "Light.direction@112");
RT_STATIC_ASSERT(sizeof(Uniforms) == 208, "Uniforms 208 B");
RT_STATIC_ASSERT(offsetof(Uniforms, maxBounces) == 24, "Uniforms.maxBounces@24");
RT_STATIC_ASSERT(offsetof(Uniforms, camera) == 32, "Uniforms.camera@32");
RT_STATIC_ASSERT(offsetof(Uniforms, previousCamera) == 96, "Uniforms.previousCamera@96");
RT_STATIC_ASSERT(offsetof(Uniforms, debugTextureMode) == 160, "Uniforms.debugTextureMode@160");
RT_STATIC_ASSERT(offsetof(Uniforms, motionSamplingHighThresholdPixels) == 204, "Uniforms@204");
RT_STATIC_ASSERT(sizeof(Material) == 64, "Material 64 B");
RT_STATIC_ASSERT(offsetof(Material, specularExponent) == 48, "Material.specularExponent@48");
RT_STATIC_ASSERT(offsetof(Material, textureFlags) == 60, "Material.textureFlags@60");
RT_STATIC_ASSERT(sizeof(rt_packed_float4x3) == 48, "packed float4x3 48 B");

#ifdef __cplusplus
}
#endif
#endif /* RT_TYPES_H */
