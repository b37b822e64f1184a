// rt_usd.h — USD layer readers for the scene ingest (the USDZ path of
// Model.init, Model.swift:87-184, and its skeleton / animation, Model.swift:346-414).
//
// The reference hands a .usdz to ModelIO (MDLAsset(url:), Model.swift:74-81) and walks the
// resulting MDLMesh / MDLSkeleton / MDLPackedJointAnimation objects.  ModelIO and the USD
// library are not in this image, so this is our own reader of the three layer encodings:
//   .usdz  zip package (stored or deflated entries); the first .usd/.usda/.usdc entry is the
//          root layer, the other entries (textures) are handed to the scene builder by name
//   .usda  text layers: prims, typed attributes (default values, timeSamples, .connect),
//          relationships, prim / property metadata (apiSchemas, interpolation, elementSize)
//   .usdc  crate binary layers (bootstrap + TOC; TOKENS / STRINGS / FIELDS / FIELDSETS / PATHS /
//          SPECS sections; LZ4 + integer-delta compression; inlined and out-of-line value reps,
//          compressed numeric arrays, list ops, time samples)
// into one in-memory Stage, then composed (load_stage): sublayers (stronger layer first), and per
// prim in namespace order its selected variants, references and payloads (LIVRPS order: local
// opinions over variants over references over payloads; a weaker opinion only fills in what is not
// authored yet), external (`@asset@</Prim>`, default prim when no path) and internal (`</Prim>`)
// arcs, paths inside the referenced subtree remapped to the referencing prim.  Assets resolve
// next to the layer that names them (inside the package for a .usdz).  .usdc layers contribute
// their subLayers and references / payloads (a reference with custom data is dropped); their
// variant specs are not read.  inherits / specializes (class arcs) are not followed.  Parity against Pixar's reader is
// unpinned (no USD asset or library in the snapshot); tests/test_usd.py pins the readers against
// files written by an independent Python writer of each encoding, and the composition against the
// same scene written flat.
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace rt {
namespace usd {

struct Value {
    enum Kind : uint8_t { kNone, kNum, kStr, kPath };
    Kind kind = kNone;
    bool array = false;
    int comps = 1;                  // numbers per element (1, 2, 3, 4, 9, 16)
    std::vector<double> num;        // all numbers, flattened (bool / int / float / tuple / matrix)
    std::vector<std::string> str;   // strings, tokens, asset paths, paths
    size_t count() const { return kind == kNum ? num.size() / (size_t)(comps > 0 ? comps : 1) : str.size(); }
};

struct Attr {
    std::string type;                       // value type name, e.g. "point3f[]", "matrix4d"
    bool uniform = false;
    bool has_default = false;
    Value value;                            // the default value
    std::vector<double> times;              // timeSamples: time codes ...
    std::vector<Value> samples;             // ... and their values
    std::vector<std::string> connections;   // .connect targets (prim path + "." + property)
    std::string interpolation;              // primvar interpolation metadata
    int element_size = 1;                   // primvar elementSize metadata
};

// a reference or payload: asset path (empty: internal) and target prim path (empty: defaultPrim)
struct Arc {
    std::string asset, path;
    bool resolved = false;   // asset is a layer id already (an arc carried out of the layer that authored it)
};

struct Prim {
    std::string name, type, path;
    // composition arcs authored on this prim (cleared once applied by load_stage)
    std::vector<Arc> references, payloads;
    std::map<std::string, std::string> variant_sel;                // variant set -> selected variant
    std::map<std::string, std::map<std::string, int>> variant_bodies;  // set -> variant -> detached prim
    int parent = -1;
    bool active = true;
    std::vector<int> children;
    std::vector<std::string> api_schemas;
    std::map<std::string, Attr> attrs;
    std::map<std::string, std::vector<std::string>> rels;
    const Attr* attr(const std::string& n) const {
        auto it = attrs.find(n);
        return it == attrs.end() ? nullptr : &it->second;
    }
    const std::vector<std::string>* rel(const std::string& n) const {
        auto it = rels.find(n);
        return it == rels.end() ? nullptr : &it->second;
    }
};

struct Stage {
    std::vector<Prim> prims;        // prims[0] is the pseudo-root "/"
    std::map<std::string, int> by_path;
    double time_codes_per_second = 24.0;
    std::string up_axis = "Y";
    std::string default_prim;
    std::vector<std::string> sublayers;   // subLayers, strongest first
    std::string layer_id;                 // the layer this stage was read from (composition)
    Stage();
    // a prim outside the namespace tree (a variant body: path "/Prim{set=variant}")
    int add_detached(const std::string& path);
    int find(const std::string& path) const {
        auto it = by_path.find(path);
        return it == by_path.end() ? -1 : it->second;
    }
    int add_prim(int parent, const std::string& name);   // returns the existing prim for a repeated path
    // depth-first pre-order of the subtree at `root` in children order, each prim once (an
    // explicit stack: a hostile file's path tree may be deep); inactive prims and their subtrees
    // are left out when active_only
    std::vector<int> preorder(int root, bool active_only) const;
};

// One file of a .usdz package.
struct PackageFile {
    std::string name;
    std::vector<uint8_t> data;
};

bool parse_usda(const char* text, size_t n, Stage& st, std::string& err);
bool parse_usdc(const uint8_t* data, size_t n, Stage& st, std::string& err);
bool read_zip(const uint8_t* data, size_t n, std::vector<PackageFile>& files, std::string& err);
// .usdz / .usda / .usdc by content; `files` receives a package's entries (empty for a bare layer)
bool load_stage(const std::string& path, Stage& st, std::vector<PackageFile>& files, std::string& err);

// LZ4 block and TfFastCompression framing (exposed for tests via the C-ABI debug hook)
bool lz4_block_decode(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_n);

}  // namespace usd
}  // namespace rt
