// rt_texture.cpp — texture ingest for the PBR texture path: the PNG decoder
// that stands in for MTKTextureLoader.newTexture(URL:options:) (SubMesh.swift:93-115).
//
// Textures are stored as RGBA8 with row 0 = the image's top row, which is how the Metal loader
// lays them out (texcoord (0, 0) = top-left; the shader flips the OBJ/USD v, Raytracing.metal:416).
// The sRGB option of the loader (base color and emission maps, SubMesh.swift:80-85) is applied
// at sampling time from the texture slot, not here.
//
// Supported: PNG, non-interlaced and Adam7, bit depths 1/2/4/8/16, greyscale, RGB, palette,
// greyscale + alpha, RGBA, tRNS transparency.  16-bit samples are rounded to 8 bits.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include <zlib.h>

#include "../../include/rt_scene.h"

namespace {

uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

struct Png {
    uint32_t w = 0, h = 0;
    int depth = 0, ctype = 0, interlace = 0;
    std::vector<uint8_t> idat, plte, trns;
};

int channels_of(int ctype) {
    switch (ctype) {
        case 0: return 1;   // grey
        case 2: return 3;   // RGB
        case 3: return 1;   // palette index
        case 4: return 2;   // grey + alpha
        case 6: return 4;   // RGBA
        default: return 0;
    }
}

bool parse(const uint8_t* d, size_t n, Png& p, std::string& err) {
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    if (n < 8 || std::memcmp(d, sig, 8) != 0) {
        err = "not a PNG file";
        return false;
    }
    size_t o = 8;
    bool have_hdr = false, end = false;
    while (o + 12 <= n && !end) {
        uint32_t len = be32(d + o);
        if (len > n - o - 12) {
            err = "truncated PNG chunk";
            return false;
        }
        const uint8_t* type = d + o + 4;
        const uint8_t* body = d + o + 8;
        uint32_t crc = be32(body + len);
        if ((uint32_t)crc32(crc32(0L, Z_NULL, 0), type, len + 4) != crc) {
            err = "PNG chunk CRC mismatch";
            return false;
        }
        if (!std::memcmp(type, "IHDR", 4)) {
            if (len != 13) {
                err = "bad IHDR";
                return false;
            }
            p.w = be32(body);
            p.h = be32(body + 4);
            p.depth = body[8];
            p.ctype = body[9];
            p.interlace = body[12];
            if (body[10] != 0 || body[11] != 0 || p.interlace > 1) {
                err = "unsupported PNG compression / filter / interlace method";
                return false;
            }
            have_hdr = true;
        } else if (!std::memcmp(type, "PLTE", 4)) {
            p.plte.assign(body, body + len);
        } else if (!std::memcmp(type, "tRNS", 4)) {
            p.trns.assign(body, body + len);
        } else if (!std::memcmp(type, "IDAT", 4)) {
            p.idat.insert(p.idat.end(), body, body + len);
        } else if (!std::memcmp(type, "IEND", 4)) {
            end = true;
        } else if (!(type[0] & 0x20)) {
            err = std::string("unknown critical PNG chunk ") + std::string((const char*)type, 4);
            return false;
        }
        o += 12 + (size_t)len;
    }
    if (!have_hdr || p.idat.empty()) {
        err = "PNG without IHDR / IDAT";
        return false;
    }
    const int ch = channels_of(p.ctype);
    const bool depth_ok = p.ctype == 0   ? (p.depth == 1 || p.depth == 2 || p.depth == 4 || p.depth == 8 || p.depth == 16)
                          : p.ctype == 3 ? (p.depth == 1 || p.depth == 2 || p.depth == 4 || p.depth == 8)
                                         : (p.depth == 8 || p.depth == 16);
    if (!ch || !depth_ok) {
        err = "unsupported PNG colour type / bit depth";
        return false;
    }
    if (p.w == 0 || p.h == 0 || (uint64_t)p.w * p.h > (1ull << 28)) {
        err = "PNG size out of range";
        return false;
    }
    if (p.ctype == 3 && (p.plte.empty() || p.plte.size() % 3)) {
        err = "palette PNG without a valid PLTE";
        return false;
    }
    return true;
}

uint8_t paeth(int a, int b, int c) {
    int pp = a + b - c;
    int pa = pp > a ? pp - a : a - pp, pb = pp > b ? pp - b : b - pp, pc = pp > c ? pp - c : c - pp;
    if (pa <= pb && pa <= pc) return (uint8_t)a;
    return (uint8_t)(pb <= pc ? b : c);
}

// Reverses the per-row filters of one (sub)image in place: rows of 1 + rowbytes bytes.
bool unfilter(uint8_t* data, size_t rows, size_t rowbytes, size_t bpp, std::string& err) {
    std::vector<uint8_t> zero(rowbytes, 0);
    const uint8_t* prev = zero.data();
    for (size_t y = 0; y < rows; ++y) {
        uint8_t* line = data + y * (rowbytes + 1);
        const int ft = line[0];
        uint8_t* r = line + 1;
        switch (ft) {
            case 0: break;
            case 1:
                for (size_t i = bpp; i < rowbytes; ++i) r[i] = (uint8_t)(r[i] + r[i - bpp]);
                break;
            case 2:
                for (size_t i = 0; i < rowbytes; ++i) r[i] = (uint8_t)(r[i] + prev[i]);
                break;
            case 3:
                for (size_t i = 0; i < rowbytes; ++i) {
                    int a = i >= bpp ? r[i - bpp] : 0;
                    r[i] = (uint8_t)(r[i] + ((a + prev[i]) >> 1));
                }
                break;
            case 4:
                for (size_t i = 0; i < rowbytes; ++i) {
                    int a = i >= bpp ? r[i - bpp] : 0, c = i >= bpp ? prev[i - bpp] : 0;
                    r[i] = (uint8_t)(r[i] + paeth(a, prev[i], c));
                }
                break;
            default:
                err = "bad PNG filter type";
                return false;
        }
        prev = r;
    }
    return true;
}

// Sample k of an unfiltered row (channels interleaved) as 0..255 / 0..65535 / palette index.
uint32_t sample_at(const uint8_t* r, size_t k, int depth) {
    if (depth == 8) return r[k];
    if (depth == 16) return (uint32_t)r[2 * k] << 8 | r[2 * k + 1];
    const size_t bit = k * (size_t)depth;
    const int shift = 8 - depth - (int)(bit & 7);
    return (r[bit >> 3] >> shift) & ((1u << depth) - 1);
}

uint8_t to8(uint32_t v, int depth) {
    if (depth == 8) return (uint8_t)v;
    if (depth == 16) return (uint8_t)((v * 255u + 32767u) / 65535u);
    return (uint8_t)(v * 255u / ((1u << depth) - 1u));
}

// Converts one unfiltered row of the (sub)image to RGBA8 pixels at out[x * xstep].
void row_to_rgba(const Png& p, const uint8_t* r, uint32_t width, uint8_t* out, size_t xstep) {
    const int ch = channels_of(p.ctype);
    for (uint32_t x = 0; x < width; ++x) {
        uint8_t* o = out + (size_t)x * xstep * 4;
        uint32_t s[4];
        for (int c = 0; c < ch; ++c) s[c] = sample_at(r, (size_t)x * ch + c, p.depth);
        if (p.ctype == 3) {
            const uint32_t i = s[0];
            const size_t np = p.plte.size() / 3;
            if (i < np) {
                o[0] = p.plte[3 * i], o[1] = p.plte[3 * i + 1], o[2] = p.plte[3 * i + 2];
            } else {
                o[0] = o[1] = o[2] = 0;
            }
            o[3] = i < p.trns.size() ? p.trns[i] : 255;
            continue;
        }
        bool key = false;   // tRNS colour key (greyscale / RGB)
        if (p.ctype == 0 && p.trns.size() >= 2) key = s[0] == ((uint32_t)p.trns[0] << 8 | p.trns[1]);
        if (p.ctype == 2 && p.trns.size() >= 6)
            key = s[0] == ((uint32_t)p.trns[0] << 8 | p.trns[1]) && s[1] == ((uint32_t)p.trns[2] << 8 | p.trns[3]) &&
                  s[2] == ((uint32_t)p.trns[4] << 8 | p.trns[5]);
        switch (p.ctype) {
            case 0: o[0] = o[1] = o[2] = to8(s[0], p.depth), o[3] = key ? 0 : 255; break;
            case 2: o[0] = to8(s[0], p.depth), o[1] = to8(s[1], p.depth), o[2] = to8(s[2], p.depth), o[3] = key ? 0 : 255; break;
            case 4: o[0] = o[1] = o[2] = to8(s[0], p.depth), o[3] = to8(s[1], p.depth); break;
            default: for (int c = 0; c < 4; ++c) o[c] = to8(s[c], p.depth); break;
        }
    }
}

}  // namespace

extern "C" {

rt_status rt_decode_png(const uint8_t* data, size_t size, uint8_t* rgba8, uint32_t* width, uint32_t* height,
                        char* err_buf, size_t err_len) {
    std::string err;
    auto fail = [&](rt_status st) {
        if (err_buf && err_len) {
            std::strncpy(err_buf, err.c_str(), err_len - 1);
            err_buf[err_len - 1] = 0;
        }
        return st;
    };
    if (!data || !width || !height) {
        err = "null argument";
        return fail(RT_ERR_INVALID_ARG);
    }
    Png p;
    if (!parse(data, size, p, err)) return fail(RT_ERR_IO);
    *width = p.w;
    *height = p.h;
    if (!rgba8) return RT_OK;   // size query
    const int ch = channels_of(p.ctype);
    const size_t bpp = std::max<size_t>(1, (size_t)ch * p.depth / 8);
    auto rowbytes = [&](uint32_t w) { return ((size_t)w * ch * p.depth + 7) / 8; };
    // the sub-images: one, or Adam7's seven passes
    static const int ax0[7] = {0, 4, 0, 2, 0, 1, 0}, ay0[7] = {0, 0, 4, 0, 2, 0, 1};
    static const int adx[7] = {8, 8, 4, 4, 2, 2, 1}, ady[7] = {8, 8, 8, 4, 4, 2, 2};
    const int passes = p.interlace ? 7 : 1;
    size_t total = 0;
    uint32_t pw[7], ph[7];
    for (int k = 0; k < passes; ++k) {
        pw[k] = p.interlace ? (p.w + adx[k] - 1 - ax0[k]) / adx[k] : p.w;
        ph[k] = p.interlace ? (p.h + ady[k] - 1 - ay0[k]) / ady[k] : p.h;
        if (p.interlace && (p.w <= (uint32_t)ax0[k] || p.h <= (uint32_t)ay0[k])) pw[k] = ph[k] = 0;
        if (pw[k] && ph[k]) total += (size_t)ph[k] * (rowbytes(pw[k]) + 1);
    }
    std::vector<uint8_t> raw(total);
    uLongf got = (uLongf)total;
    if (uncompress(raw.data(), &got, p.idat.data(), (uLong)p.idat.size()) != Z_OK || got != total) {
        err = "corrupt PNG image data";
        return fail(RT_ERR_IO);
    }
    size_t off = 0;
    for (int k = 0; k < passes; ++k) {
        if (!pw[k] || !ph[k]) continue;
        const size_t rb = rowbytes(pw[k]);
        if (!unfilter(raw.data() + off, ph[k], rb, bpp, err)) return fail(RT_ERR_IO);
        for (uint32_t y = 0; y < ph[k]; ++y) {
            const uint8_t* r = raw.data() + off + (size_t)y * (rb + 1) + 1;
            const size_t oy = p.interlace ? (size_t)ay0[k] + (size_t)y * ady[k] : y;
            const size_t ox = p.interlace ? (size_t)ax0[k] : 0;
            row_to_rgba(p, r, pw[k], rgba8 + (oy * p.w + ox) * 4, p.interlace ? (size_t)adx[k] : 1);
        }
        off += (size_t)ph[k] * (rb + 1);
    }
    return RT_OK;
}

rt_status rt_write_png(const char* path, const uint8_t* rgba8, uint32_t width, uint32_t height) {
    if (!path || !rgba8 || width == 0 || height == 0) return RT_ERR_INVALID_ARG;
    const size_t row = (size_t)width * 4;
    std::vector<uint8_t> raw((row + 1) * height);
    for (uint32_t y = 0; y < height; ++y) {
        raw[y * (row + 1)] = 0;   // filter: none
        std::memcpy(&raw[y * (row + 1) + 1], rgba8 + y * row, row);
    }
    uLongf zlen = compressBound((uLong)raw.size());
    std::vector<uint8_t> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK) return RT_ERR_IO;
    FILE* f = std::fopen(path, "wb");
    if (!f) return RT_ERR_IO;
    auto put32 = [](uint8_t* p, uint32_t v) { p[0] = v >> 24, p[1] = v >> 16, p[2] = v >> 8, p[3] = v; };
    auto chunk = [&](const char* type, const uint8_t* body, uint32_t len) {
        uint8_t hdr[8];
        put32(hdr, len);
        std::memcpy(hdr + 4, type, 4);
        uLong crc = crc32(0L, Z_NULL, 0);
        crc = crc32(crc, hdr + 4, 4);
        if (len) crc = crc32(crc, body, len);
        uint8_t tail[4];
        put32(tail, (uint32_t)crc);
        std::fwrite(hdr, 1, 8, f);
        if (len) std::fwrite(body, 1, len, f);
        std::fwrite(tail, 1, 4, f);
    };
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    std::fwrite(sig, 1, 8, f);
    uint8_t ihdr[13];
    put32(ihdr, width);
    put32(ihdr + 4, height);
    ihdr[8] = 8, ihdr[9] = 6, ihdr[10] = 0, ihdr[11] = 0, ihdr[12] = 0;
    chunk("IHDR", ihdr, 13);
    chunk("IDAT", z.data(), (uint32_t)zlen);
    chunk("IEND", nullptr, 0);
    const bool ok = std::ferror(f) == 0;
    return std::fclose(f) == 0 && ok ? RT_OK : RT_ERR_IO;
}

}  // extern "C"
