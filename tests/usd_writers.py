"""Test-only writers of the three USD encodings rt_usd.cpp reads (.usda text, .usdc crate,
.usdz package), written from the published format descriptions independently of the C++ reader:
a scene described once as Python prims is written in each encoding, and the scene the library
builds from each must agree (tests/test_usd.py).

Crate layout written here (Pixar's crateFile.cpp, version 0.8.0): 88-byte bootstrap ("PXR-USDC",
version, TOC offset), sections TOKENS (count, sizes, LZ4 of NUL-separated tokens), STRINGS,
FIELDS (compressed token indices + LZ4 of 64-bit value reps), FIELDSETS (compressed field
indices, ~0 terminated), PATHS (compressed path indexes / element tokens / sibling jumps, depth
first), SPECS (compressed path / fieldset / spec-type indexes); TOC = count + (name[16], start,
size).  Integer blocks use the delta coding (common delta, 2-bit codes, 8/16/32-bit deltas);
LZ4 blocks come from the small greedy compressor below (TfFastCompression framing: a leading
chunk-count byte of 0)."""
import io
import math
import struct
import zipfile
import zlib
from collections import Counter

# ---- scene description -------------------------------------------------------------------------
# prim: dict(path, type, api=[...], attrs=[Attr...], rels={name: [paths]})
# Attr: dict(name, type, value=None, uniform=False, interpolation=None, element_size=None,
#            samples=None ({time: value}), connect=None ([paths]))
# values: numbers, tuples, lists of numbers / tuples, ("token", s), ("asset", s), matrices as
# 4-tuples of 4-tuples (rows), quats as (w, x, y, z)


def _fmt(v):
    if isinstance(v, tuple) and len(v) == 2 and v[0] in ("token", "asset"):
        return ('"%s"' % v[1]) if v[0] == "token" else ("@%s@" % v[1])
    if isinstance(v, (list,)):
        return "[" + ", ".join(_fmt(x) for x in v) + "]"
    if isinstance(v, tuple):
        return "(" + ", ".join(_fmt(x) for x in v) + ")"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, int):
        return str(v)
    return repr(float(v))


def write_usda(prims, tcps=24.0, up_axis="Y"):
    out = ["#usda 1.0", "(", '    upAxis = "%s"' % up_axis, "    timeCodesPerSecond = %s" % tcps,
           '    doc = """test layer"""', ")", ""]
    children = {}
    for p in prims:
        parent = p["path"].rsplit("/", 1)[0] or "/"
        children.setdefault(parent, []).append(p)

    def emit(p, ind):
        pad = "    " * ind
        meta = ""
        if p.get("api"):
            meta = ' (\n%s    prepend apiSchemas = [%s]\n%s)' % (pad, ", ".join('"%s"' % a for a in p["api"]), pad)
        name = p["path"].rsplit("/", 1)[1]
        out.append('%sdef %s "%s"%s' % (pad, p.get("type", ""), name, meta) if p.get("type")
                   else '%sdef "%s"%s' % (pad, name, meta))
        out.append(pad + "{")
        for a in p.get("attrs", []):
            pre = pad + "    " + ("uniform " if a.get("uniform") else "")
            md = []
            if a.get("interpolation"):
                md.append('interpolation = "%s"' % a["interpolation"])
            if a.get("element_size"):
                md.append("elementSize = %d" % a["element_size"])
            mds = (" (\n%s        %s\n%s    )" % (pad, "\n        ".join(md), pad)) if md else ""
            if a.get("connect"):
                out.append("%s%s %s.connect = %s" % (pre, a["type"], a["name"],
                                                     ("<%s>" % a["connect"][0]) if len(a["connect"]) == 1
                                                     else "[" + ", ".join("<%s>" % c for c in a["connect"]) + "]"))
            if a.get("samples") is not None:
                body = ",\n".join("%s        %s: %s" % (pad, _fmt(t), _fmt(v)) for t, v in sorted(a["samples"].items()))
                out.append("%s%s %s.timeSamples = {\n%s,\n%s    }" % (pre, a["type"], a["name"], body, pad))
            if a.get("value") is not None:
                out.append("%s%s %s = %s%s" % (pre, a["type"], a["name"], _fmt(a["value"]), mds))
            elif not a.get("connect") and a.get("samples") is None:
                out.append("%s%s %s%s" % (pre, a["type"], a["name"], mds))
        for rel, targets in p.get("rels", {}).items():
            tv = ("<%s>" % targets[0]) if len(targets) == 1 else "[" + ", ".join("<%s>" % t for t in targets) + "]"
            out.append("%s    rel %s = %s" % (pad, rel, tv))
        for c in children.get(p["path"], []):
            out.append("")
            emit(c, ind + 1)
        out.append(pad + "}")

    for p in children.get("/", []):
        emit(p, 0)
        out.append("")
    return "\n".join(out).encode()


# ---- LZ4 block (greedy) + TfFastCompression framing ---------------------------------------------
def lz4_compress(src):
    src = bytes(src)
    n = len(src)
    out = bytearray()
    table = {}
    i = anchor = 0

    def emit(lit, off, ml):
        ln = len(lit)
        tok = (min(ln, 15) << 4) | (min(ml - 4, 15) if ml else 0)
        out.append(tok)
        if ln >= 15:
            r = ln - 15
            while r >= 255:
                out.append(255)
                r -= 255
            out.append(r)
        out.extend(lit)
        if ml:
            out.extend(struct.pack("<H", off))
            if ml - 4 >= 15:
                r = ml - 4 - 15
                while r >= 255:
                    out.append(255)
                    r -= 255
                out.append(r)

    while i + 12 < n:
        key = src[i:i + 4]
        j = table.get(key)
        table[key] = i
        if j is not None and i - j <= 65535:
            ml = 4
            while i + ml < n - 5 and src[j + ml] == src[i + ml]:
                ml += 1
            emit(src[anchor:i], i - j, ml)
            i += ml
            anchor = i
        else:
            i += 1
    emit(src[anchor:], 0, 0)
    return bytes(out)


def fast_compress(src):
    return b"\x00" + lz4_compress(src)


def encode_ints(vals, bits=32):
    """Usd_IntegerCompression: deltas, the most common one as the header, 2-bit codes."""
    small, medium = (1, 2) if bits == 32 else (2, 4)
    big = 4 if bits == 32 else 8
    fmt = {1: "<b", 2: "<h", 4: "<i", 8: "<q"}
    deltas, prev = [], 0
    half = 1 << (bits - 1)
    for v in vals:   # two's-complement deltas (uint32 fieldset terminators wrap)
        deltas.append((int(v) - prev + half) % (2 * half) - half)
        prev = int(v)
    common = Counter(deltas).most_common(1)[0][0] if deltas else 0
    codes = bytearray((len(deltas) * 2 + 7) // 8)
    payload = bytearray()
    for i, d in enumerate(deltas):
        if d == common:
            c = 0
        elif -(1 << (8 * small - 1)) <= d < (1 << (8 * small - 1)):
            c, sz = 1, small
        elif -(1 << (8 * medium - 1)) <= d < (1 << (8 * medium - 1)):
            c, sz = 2, medium
        else:
            c, sz = 3, big
        codes[i // 4] |= c << (2 * (i % 4))
        if c:
            payload += struct.pack(fmt[sz], d)
    raw = struct.pack("<i" if bits == 32 else "<q", common) + bytes(codes) + bytes(payload)
    comp = fast_compress(raw)
    return struct.pack("<Q", len(comp)) + comp


# ---- crate writer -------------------------------------------------------------------------------
T_BOOL, T_INT, T_FLOAT, T_DOUBLE, T_HALF = 1, 3, 8, 9, 7
T_TOKEN, T_ASSET, T_MATRIX4D, T_QUATF = 11, 12, 15, 17
T_VEC2F, T_VEC3F, T_VEC3H = 20, 24, 25
T_TOKENLISTOP, T_PATHLISTOP, T_TOKENVECTOR = 32, 34, 41
T_SPECIFIER, T_VARIABILITY, T_TIMESAMPLES, T_DOUBLEVECTOR = 42, 44, 46, 48
T_REFERENCELISTOP, T_STRINGVECTOR = 35, 50
T_STRINGLISTOP, T_VARIANTSELECTIONMAP = 33, 45
ARRAY, INLINE, COMPRESSED = 1 << 63, 1 << 62, 1 << 61

_TYPE_OF = {
    "point3f": T_VEC3F, "normal3f": T_VEC3F, "color3f": T_VEC3F, "float3": T_VEC3F, "vector3f": T_VEC3F,
    "texCoord2f": T_VEC2F, "float2": T_VEC2F, "half3": T_VEC3H, "quatf": T_QUATF, "matrix4d": T_MATRIX4D,
    "int": T_INT, "float": T_FLOAT, "double": T_DOUBLE, "token": T_TOKEN, "asset": T_ASSET, "bool": T_BOOL,
}


class CrateWriter:
    def __init__(self, jumps_hook=None):
        self.tokens, self.tok_index = [], {}
        self.strings, self.str_index = [], {}   # STRINGS: string index -> token index
        self.data = bytearray(b"\0" * 88)   # bootstrap, patched at the end
        self.jumps_hook = jumps_hook          # tests: rewrites the PATHS sibling-jump table

    def tok(self, s):
        if s not in self.tok_index:
            self.tok_index[s] = len(self.tokens)
            self.tokens.append(s)
        return self.tok_index[s]

    def string(self, s):
        if s not in self.str_index:
            self.str_index[s] = len(self.strings)
            self.strings.append(self.tok(s))
        return self.str_index[s]

    def string_vector(self, strs):
        off = self.here()
        self.data += struct.pack("<Q", len(strs)) + b"".join(struct.pack("<I", self.string(x)) for x in strs)
        return self.rep(T_STRINGVECTOR, off)

    def reference_list_op(self, refs, path_idx, appended=()):
        """prepended (and appended) SdfReferences: asset (string index), prim path (path index),
        layer offset (offset 0, scale 1), empty custom data; the lists in file order (explicit,
        added, prepended, appended)"""
        off = self.here()
        self.data += bytes([(1 << 5 if refs else 0) | (1 << 6 if appended else 0)])
        for items in (refs, appended):
            if not items:
                continue
            self.data += struct.pack("<Q", len(items))
            for asset, path in items:
                # "" (the asset's default prim): an index past the path table reads as the empty path
                self.data += struct.pack("<II", self.string(asset), path_idx[path] if path else 0xffffffff)
                self.data += struct.pack("<dd", 0.0, 1.0)
                self.data += struct.pack("<Q", 0)
        return self.rep(T_REFERENCELISTOP, off)

    def here(self):
        return len(self.data)

    def variant_selection(self, sel):
        """SdfVariantSelectionMap: count, then (set, variant) string indexes"""
        off = self.here()
        self.data += struct.pack("<Q", len(sel))
        for k, v in sorted(sel.items()):
            self.data += struct.pack("<II", self.string(k), self.string(v))
        return self.rep(T_VARIANTSELECTIONMAP, off)

    def rep(self, t, payload, flags=0):
        return flags | (t << 48) | payload

    # ---- values -------------------------------------------------------------------------------
    def value(self, type_name, v):
        base = type_name[:-2] if type_name.endswith("[]") else type_name
        arr = type_name.endswith("[]")
        t = _TYPE_OF[base]
        if t in (T_TOKEN, T_ASSET):
            if not arr:
                return self.rep(t, self.tok(v[1]), INLINE)
            off = self.here()
            self.data += struct.pack("<Q", len(v)) + b"".join(struct.pack("<I", self.tok(x[1])) for x in v)
            return self.rep(t, off, ARRAY)
        if not arr:
            return self.scalar(t, v)
        return self.array(t, v)

    def scalar(self, t, v):
        if t == T_INT:
            return self.rep(t, v & 0xffffffff, INLINE)
        if t == T_FLOAT:
            return self.rep(t, struct.unpack("<I", struct.pack("<f", v))[0], INLINE)
        if t == T_DOUBLE:
            f = struct.unpack("<f", struct.pack("<f", v))[0]
            if f == v:
                return self.rep(t, struct.unpack("<I", struct.pack("<f", v))[0], INLINE)
            off = self.here()
            self.data += struct.pack("<d", v)
            return self.rep(t, off)
        if t == T_MATRIX4D:
            flat = [x for row in v for x in row]
            diag = all(flat[i] == 0 for i in range(16) if i % 5) and all(float(int(flat[i])) == flat[i] and
                                                                         -128 <= flat[i] < 128 for i in (0, 5, 10, 15))
            if diag:
                p = 0
                for k, i in enumerate((0, 5, 10, 15)):
                    p |= (int(flat[i]) & 0xff) << (8 * k)
                return self.rep(t, p, INLINE)
            off = self.here()
            self.data += struct.pack("<16d", *flat)
            return self.rep(t, off)
        if t in (T_VEC3F, T_VEC2F):
            if all(float(int(x)) == x and -128 <= x < 128 for x in v):
                p = 0
                for k, x in enumerate(v):
                    p |= (int(x) & 0xff) << (8 * k)
                return self.rep(t, p, INLINE)
            off = self.here()
            self.data += struct.pack("<%df" % len(v), *v)
            return self.rep(t, off)
        raise ValueError(t)

    def array(self, t, v):
        off = self.here()
        self.data += struct.pack("<Q", len(v))
        if t == T_INT:
            if len(v) >= 16:
                self.data += encode_ints(v)
                return self.rep(t, off, ARRAY | COMPRESSED)
            self.data += struct.pack("<%di" % len(v), *v)
            return self.rep(t, off, ARRAY)
        if t == T_FLOAT:
            if len(v) >= 16:
                if all(float(int(x)) == x for x in v):   # 'i': stored as integers
                    self.data += b"i" + encode_ints([int(x) for x in v])
                else:                                       # 't': lookup table + indexes
                    lut = sorted(set(v))
                    self.data += b"t" + struct.pack("<I", len(lut)) + struct.pack("<%df" % len(lut), *lut)
                    self.data += encode_ints([lut.index(x) for x in v])
                return self.rep(t, off, ARRAY | COMPRESSED)
            self.data += struct.pack("<%df" % len(v), *v)
            return self.rep(t, off, ARRAY)
        if t in (T_VEC3F, T_VEC2F):
            flat = [x for e in v for x in e]
            self.data += struct.pack("<%df" % len(flat), *flat)
        elif t == T_VEC3H:
            flat = [x for e in v for x in e]
            self.data += struct.pack("<%de" % len(flat), *flat)
        elif t == T_QUATF:   # GfQuatf memory order: imaginary (i, j, k), then real
            flat = [x for (w, i, j, k) in v for x in (i, j, k, w)]
            self.data += struct.pack("<%df" % len(flat), *flat)
        elif t == T_MATRIX4D:
            flat = [x for m in v for row in m for x in row]
            self.data += struct.pack("<%dd" % len(flat), *flat)
        else:
            raise ValueError(t)
        return self.rep(t, off, ARRAY)

    def token_vector(self, toks):
        off = self.here()
        self.data += struct.pack("<Q", len(toks)) + b"".join(struct.pack("<I", self.tok(x)) for x in toks)
        return self.rep(T_TOKENVECTOR, off)

    def list_op(self, t, idx):
        off = self.here()
        self.data += bytes([1 << 5])   # prepended items only
        self.data += struct.pack("<Q", len(idx)) + b"".join(struct.pack("<I", i) for i in idx)
        return self.rep(t, off)

    def time_samples(self, type_name, samples):
        times = sorted(samples)
        reps = [self.value(type_name, samples[t]) for t in times]
        toff = self.here()
        self.data += struct.pack("<Q", len(times)) + struct.pack("<%dd" % len(times), *times)
        times_rep = self.rep(T_DOUBLEVECTOR, toff)
        off = self.here()
        self.data += struct.pack("<q", 16) + struct.pack("<Q", times_rep)
        self.data += struct.pack("<q", 16 + 8 * len(reps)) + struct.pack("<Q", len(reps))
        self.data += b"".join(struct.pack("<Q", r) for r in reps)
        return self.rep(T_TIMESAMPLES, off)

    # ---- layer ----------------------------------------------------------------------------------
    def write(self, prims, tcps=24.0, up_axis="Y", sublayers=None):
        """prims: dicts with "path" (a variant body is "<prim>{set=variant}", its children
        "<prim>{set=variant}/Child"), "type", "attrs", "rels", "api", "refs", "variant_sel"
        ({set: variant}) and "variant_sets" ({set: [variants]}: the "{set=}" variant set specs and
        the prim's variantSetNames)"""
        def split(path):   # (parent path, element token)
            if path.endswith("}") and path.rfind("{") > path.rfind("/"):
                return path[:path.rfind("{")], path[path.rfind("{"):]
            return path.rsplit("/", 1)[0] or "/", path.rsplit("/", 1)[1]

        prims = list(prims)
        for p in list(prims):   # variant set specs "<prim>{set=}"
            for vset, names in p.get("variant_sets", {}).items():
                prims.append({"path": p["path"] + "{" + vset + "=}", "variant_children": names})
        kids = {"/": []}
        props = {}
        for p in prims:
            parent = split(p["path"])[0]
            kids.setdefault(parent, []).append(p["path"])
            kids.setdefault(p["path"], [])
            props[p["path"]] = [a["name"] for a in p.get("attrs", [])] + list(p.get("rels", {}))
        by = {p["path"]: p for p in prims}
        # depth-first path list: prim, its properties, its children (jumps point at siblings)
        order = []   # (path, element token, is_property, has_child, sibling_path)

        def visit(path, sib):
            name = split(path)[1] if path != "/" else ""
            entries = [(path + "." + pr, pr) for pr in props.get(path, [])] + [(c, None) for c in kids.get(path, [])]
            order.append([path, name, False, bool(entries), sib])
            for k, (pp, pr) in enumerate(entries):
                nxt = entries[k + 1][0] if k + 1 < len(entries) else None
                if pr is not None:
                    order.append([pp, pr, True, False, nxt])
                else:
                    visit(pp, nxt)

        visit("/", None)
        index_of = {e[0]: i for i, e in enumerate(order)}
        path_idx = {e[0]: i for i, e in enumerate(order)}   # path table index = DFS position
        fields, field_index, fieldsets, specs = [], {}, [], []

        def field(name, rep):
            key = (self.tok(name), rep)
            if key not in field_index:
                field_index[key] = len(fields)
                fields.append(key)
            return field_index[key]

        def spec(path, fl, kind):
            specs.append((path_idx[path], len(fieldsets), kind))
            fieldsets.extend(fl + [0xffffffff])

        root_kids = [c.rsplit("/", 1)[1] for c in kids["/"]]
        spec("/", [field("primChildren", self.token_vector(root_kids)),
                   field("upAxis", self.rep(T_TOKEN, self.tok(up_axis), INLINE)),
                   field("timeCodesPerSecond", self.scalar(T_DOUBLE, tcps))] +
             ([field("subLayers", self.string_vector(sublayers))] if sublayers else []), 7)
        for p in prims:
            if "variant_children" in p:   # a variant set spec
                spec(p["path"], [field("variantChildren", self.token_vector(p["variant_children"]))], 11)
                continue
            fl = [field("specifier", self.rep(T_SPECIFIER, 0, INLINE))]
            if p.get("type"):
                fl.append(field("typeName", self.rep(T_TOKEN, self.tok(p["type"]), INLINE)))
            real = [split(c)[1] for c in kids[p["path"]] if not split(c)[1].startswith("{")]
            if real:
                fl.append(field("primChildren", self.token_vector(real)))
            if p.get("variant_sets"):
                fl.append(field("variantSetNames", self.list_op(T_STRINGLISTOP,
                                                                [self.string(x) for x in p["variant_sets"]])))
            if p.get("variant_sel"):
                fl.append(field("variantSelection", self.variant_selection(p["variant_sel"])))
            if props[p["path"]]:
                fl.append(field("properties", self.token_vector(props[p["path"]])))
            if p.get("api"):
                fl.append(field("apiSchemas", self.list_op(T_TOKENLISTOP, [self.tok(a) for a in p["api"]])))
            if p.get("refs") or p.get("refs_appended"):   # [(asset, target prim path in this layer's path table)]
                fl.append(field("references", self.reference_list_op(p.get("refs") or [], path_idx,
                                                                     p.get("refs_appended") or [])))
            spec(p["path"], fl, p.get("kind", 10 if p["path"].endswith("}") else 6))
            for a in p.get("attrs", []):
                fl = [field("typeName", self.rep(T_TOKEN, self.tok(a["type"]), INLINE))]
                if a.get("uniform"):
                    fl.append(field("variability", self.rep(T_VARIABILITY, 1, INLINE)))
                if a.get("interpolation"):
                    fl.append(field("interpolation", self.rep(T_TOKEN, self.tok(a["interpolation"]), INLINE)))
                if a.get("element_size"):
                    fl.append(field("elementSize", self.rep(T_INT, a["element_size"], INLINE)))
                if a.get("value") is not None:
                    fl.append(field("default", self.value(a["type"], a["value"])))
                if a.get("samples") is not None:
                    fl.append(field("timeSamples", self.time_samples(a["type"], a["samples"])))
                if a.get("connect"):
                    fl.append(field("connectionPaths", self.list_op(T_PATHLISTOP, [path_idx[c] for c in a["connect"]])))
                spec(p["path"] + "." + a["name"], fl, 1)
            for rel, targets in p.get("rels", {}).items():
                spec(p["path"] + "." + rel, [field("targetPaths", self.list_op(T_PATHLISTOP, [path_idx[t] for t in targets]))], 8)
        for e in order:   # element tokens first, so every token exists before TOKENS is written
            self.tok(e[1])
        sections = []

        def section(name, body):
            start = self.here()
            self.data += body
            sections.append((name, start, len(body)))

        blob = b"".join(t.encode() + b"\0" for t in self.tokens)
        comp = fast_compress(blob)
        section("TOKENS", struct.pack("<QQQ", len(self.tokens), len(blob), len(comp)) + comp)
        section("STRINGS", struct.pack("<Q", len(self.strings)) + b"".join(struct.pack("<I", t) for t in self.strings))
        reps = b"".join(struct.pack("<Q", r) for _, r in fields)
        rc = fast_compress(reps)
        section("FIELDS", struct.pack("<Q", len(fields)) + encode_ints([t for t, _ in fields]) + struct.pack("<Q", len(rc)) + rc)
        section("FIELDSETS", struct.pack("<Q", len(fieldsets)) + encode_ints(fieldsets))
        jumps = []
        for i, e in enumerate(order):
            has_child, sib = e[3], e[4]
            if has_child and sib is not None:
                jumps.append(index_of[sib] - i)
            elif has_child:
                jumps.append(-1)
            elif sib is not None:
                jumps.append(0)
            else:
                jumps.append(-2)
        if self.jumps_hook is not None:
            jumps = self.jumps_hook(jumps)
        elems = [0 if i == 0 else (-self.tok(e[1]) if e[2] else self.tok(e[1])) for i, e in enumerate(order)]
        section("PATHS", struct.pack("<QQ", len(order), len(order)) + encode_ints(list(range(len(order)))) +
                encode_ints(elems) + encode_ints(jumps))
        section("SPECS", struct.pack("<Q", len(specs)) + encode_ints([s[0] for s in specs]) +
                encode_ints([s[1] for s in specs]) + encode_ints([s[2] for s in specs]))
        toc = self.here()
        self.data += struct.pack("<Q", len(sections))
        for name, start, size in sections:
            self.data += name.encode().ljust(16, b"\0") + struct.pack("<QQ", start, size)
        self.data[0:24] = b"PXR-USDC" + bytes([0, 8, 0, 0, 0, 0, 0, 0]) + struct.pack("<Q", toc)
        return bytes(self.data)


def write_usdc(prims, tcps=24.0, up_axis="Y", sublayers=None):
    return CrateWriter().write(prims, tcps, up_axis, sublayers)


def write_usdz(layer_name, layer_bytes, extra=(), deflate=False):
    buf = io.BytesIO()
    mode = zipfile.ZIP_DEFLATED if deflate else zipfile.ZIP_STORED
    with zipfile.ZipFile(buf, "w", mode) as z:
        z.writestr(layer_name, layer_bytes)
        for name, data in extra:
            z.writestr(name, data)
    return buf.getvalue()


def png_rgba(w, h, pixels):
    """Minimal 8-bit RGBA PNG (filter 0 rows)."""
    raw = b"".join(b"\0" + bytes(pixels[y * w * 4:(y + 1) * w * 4]) for y in range(h))

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xffffffff)

    return (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 6, 0, 0, 0)) +
            chunk(b"IDAT", zlib.compress(raw)) + chunk(b"IEND", b""))


def half_round(x):
    return struct.unpack("<e", struct.pack("<e", x))[0]


def f32(x):
    return struct.unpack("<f", struct.pack("<f", x))[0]


def quat_from_axis_angle(axis, angle):
    s = math.sin(angle / 2)
    n = math.sqrt(sum(a * a for a in axis))
    return (math.cos(angle / 2),) + tuple(a / n * s for a in axis)
