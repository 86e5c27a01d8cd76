// pt_texture.cpp -- host image I/O: the env-map texture of config 4 (Radiance RGBE .hdr decoding)
// and the output image (24-bit BMP writing, pt_write_bmp at the end of this file).
//
// Replaces LoadTexture (asset_loading.cpp:9-16): stbi_loadf(path, &W, &H, &C, 0) with
// stbi_set_flip_vertically_on_load(true).  stb_image v2.26 (vendored by the reference,
// stb_image.h:6992-7195) is restated here, not linked:
//   * first line "#?RADIANCE" or "#?RGBE"; header lines up to an empty line, one of them must be
//     "FORMAT=32-bit_rle_rgbe"; then "-Y <H> +X <W>" (the only orientation stb accepts);
//   * width < 8 or >= 32768: flat RGBE quadruples; otherwise per scanline either the new RLE form
//     (2, 2, W>>8, W&255, then four channel planes of runs (count > 128: count-128 copies of one
//     byte) and dumps) or -- if a scanline does not start with that marker -- the whole image is
//     read flat from there, restarting at pixel 1 of row 0 (stb's `goto main_decode_loop`);
//   * RGBE -> f32: e == 0 gives 0, else c * 2^(e-136) for c in {r,g,b} (exact in f32);
//   * 3 components; rows flipped so that row 0 is the bottom of the image.
// Deviation: a truncated file is an error here (stb reads zeros past the end).  Checked bit for
// bit against stb_image compiled from the reference's sources (tests/test_texture.py).
#include "../../include/pt_mi355.h"
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

namespace {

struct Reader {
    const unsigned char* p;
    size_t n, i;
    bool eof() const { return i >= n; }
    int get8() { return i < n ? p[i++] : -1; }
};

// stbi__hdr_gettoken (stb_image.h:7014-7034): one line without its '\n', at most 1023 chars
void gettoken(Reader& r, char* buf)
{
    int len = 0;
    int c = r.get8();
    while (c >= 0 && c != '\n') {
        buf[len++] = (char)c;
        if (len == 1023) {
            while (!r.eof() && r.get8() != '\n') {
            }
            break;
        }
        c = r.get8();
    }
    buf[len] = 0;
}

// stbi__hdr_convert (stb_image.h:7036-7062), 3 components
void convert(float* out, const unsigned char* rgbe)
{
    if (rgbe[3] != 0) {
        const float f1 = (float)ldexp(1.0f, (int)rgbe[3] - (128 + 8));
        out[0] = (float)rgbe[0] * f1;
        out[1] = (float)rgbe[1] * f1;
        out[2] = (float)rgbe[2] * f1;
    } else {
        out[0] = out[1] = out[2] = 0.0f;
    }
}

// returns nullptr on success, else an error message
const char* decode(Reader& r, std::vector<float>& img, int& W, int& H)
{
    char buf[1024];
    gettoken(r, buf);
    if (strcmp(buf, "#?RADIANCE") != 0 && strcmp(buf, "#?RGBE") != 0) return "not a Radiance HDR file";
    bool valid = false;
    for (;;) {
        if (r.eof()) return "truncated HDR header";
        gettoken(r, buf);
        if (buf[0] == 0) break;
        if (strcmp(buf, "FORMAT=32-bit_rle_rgbe") == 0) valid = true;
    }
    if (!valid) return "unsupported HDR format (FORMAT=32-bit_rle_rgbe required)";
    gettoken(r, buf);
    if (strncmp(buf, "-Y ", 3) != 0) return "unsupported HDR data layout";
    char* t = buf + 3;
    const long h = strtol(t, &t, 10);
    while (*t == ' ') ++t;
    if (strncmp(t, "+X ", 3) != 0) return "unsupported HDR data layout";
    const long w = strtol(t + 3, nullptr, 10);
    if (w <= 0 || h <= 0 || w > (1 << 24) || h > (1 << 24) || (double)w * (double)h > (double)(1u << 30))
        return "invalid HDR dimensions";
    W = (int)w;
    H = (int)h;
    img.assign((size_t)W * H * 3, 0.0f);

    auto flat_from = [&](int j0, int i0) -> const char* {
        for (int j = j0; j < H; ++j)
            for (int i = (j == j0 ? i0 : 0); i < W; ++i) {
                if (r.n - r.i < 4) return "truncated HDR pixel data";
                convert(&img[((size_t)j * W + i) * 3], r.p + r.i);
                r.i += 4;
            }
        return nullptr;
    };
    if (W < 8 || W >= 32768) return flat_from(0, 0);

    std::vector<unsigned char> scan((size_t)W * 4);
    for (int j = 0; j < H; ++j) {
        if (r.n - r.i < 4) return "truncated HDR scanline";
        const int c1 = r.p[r.i], c2 = r.p[r.i + 1], len0 = r.p[r.i + 2];
        if (c1 != 2 || c2 != 2 || (len0 & 0x80)) {
            // not run-length encoded: these 4 bytes are pixel (0, 0), then everything flat
            convert(&img[0], r.p + r.i);
            r.i += 4;
            return flat_from(0, 1);
        }
        const int len = (len0 << 8) | r.p[r.i + 3];
        r.i += 4;
        if (len != W) return "invalid decoded HDR scanline length";
        for (int k = 0; k < 4; ++k) {
            int i = 0;
            while (W - i > 0) {
                const int nleft = W - i;
                int count = r.get8();
                if (count < 0) return "truncated HDR RLE data";
                if (count > 128) {
                    const int value = r.get8();
                    if (value < 0) return "truncated HDR RLE data";
                    count -= 128;
                    if (count > nleft) return "bad RLE data in HDR";
                    for (int z = 0; z < count; ++z) scan[(size_t)(i++) * 4 + k] = (unsigned char)value;
                } else {
                    if (count > nleft) return "bad RLE data in HDR";
                    if ((size_t)count > r.n - r.i) return "truncated HDR RLE data";
                    for (int z = 0; z < count; ++z) scan[(size_t)(i++) * 4 + k] = r.p[r.i++];
                }
            }
        }
        for (int i = 0; i < W; ++i) convert(&img[((size_t)j * W + i) * 3], &scan[(size_t)i * 4]);
    }
    return nullptr;
}

}  // namespace

int pt_internal_fail(int code, const char* fmt, ...);   // pt_capi.cpp: sets pt_last_error()

extern "C" {

int pt_decode_hdr(const void* bytes, size_t nbytes, pt_texture* out)
{
    if (!out || (!bytes && nbytes)) {
        return pt_internal_fail(PT_EINVAL, "null argument");
    }
    memset(out, 0, sizeof(*out));
    Reader r{(const unsigned char*)bytes, nbytes, 0};
    std::vector<float> img;
    int W = 0, H = 0;
    if (const char* e = decode(r, img, W, H)) {
        return pt_internal_fail(PT_EINVAL, "%s", e);
    }
    float* data = (float*)malloc(img.size() * sizeof(float));
    if (!data) {
        return pt_internal_fail(PT_ENOMEM, "out of host memory");
    }
    // stbi__vertical_flip (stbi_set_flip_vertically_on_load(true), asset_loading.cpp:12)
    const size_t row = (size_t)W * 3;
    for (int j = 0; j < H; ++j) memcpy(data + (size_t)(H - 1 - j) * row, &img[(size_t)j * row], row * sizeof(float));
    out->data = data;
    out->width = W;
    out->height = H;
    out->components = 3;
    return PT_OK;
}

int pt_load_texture(const char* path, pt_texture* out)
{
    if (!path || !out) {
        return pt_internal_fail(PT_EINVAL, "null argument");
    }
    FILE* f = fopen(path, "rb");
    if (!f) {
        return pt_internal_fail(PT_EINVAL, "cannot open %s", path);
    }
    std::vector<unsigned char> bytes;
    unsigned char chunk[1 << 16];
    size_t got;
    while ((got = fread(chunk, 1, sizeof(chunk), f)) > 0) bytes.insert(bytes.end(), chunk, chunk + got);
    fclose(f);
    return pt_decode_hdr(bytes.data(), bytes.size(), out);
}

// WriteImage (asset_loading.cpp:48-54) = stbi_write_bmp of stb_image_write v1.15
// (stb_image_write.h:348-521), restated: a 54-byte header ('BM', file size, 0, 0, 54 | 40, w, h,
// 1 plane, 24 bpp, six zero words), then the rows bottom-up, pixels as B, G, R, each row padded
// to 4 bytes with zeros.  1/2 components: grey (alpha ignored); 3: RGB; 4: RGB composited over
// the pink (255, 0, 255) background by alpha with integer arithmetic (opaque pixels unchanged).
// Checked byte for byte against stb compiled from the reference's sources (tests/test_bmp.py).
int pt_write_bmp(const char* path, int32_t w, int32_t h, int32_t comp, const void* data)
{
    if (!path || (!data && w > 0 && h > 0)) return pt_internal_fail(PT_EINVAL, "null argument");
    if (w < 0 || h < 0) return pt_internal_fail(PT_EINVAL, "invalid size %dx%d", w, h);
    if (comp < 1 || comp > 4) return pt_internal_fail(PT_EINVAL, "components must be 1..4, got %d", comp);
    if ((int64_t)w * h > (int64_t)1 << 30) return pt_internal_fail(PT_EINVAL, "image too large");
    const int pad = (-w * 3) & 3;
    const uint32_t row_bytes = (uint32_t)w * 3u + (uint32_t)pad;
    std::vector<unsigned char> f;
    f.reserve(54 + (size_t)row_bytes * h);
    auto u8 = [&](uint32_t v) { f.push_back((unsigned char)v); };
    auto u16 = [&](uint32_t v) { u8(v & 0xff); u8((v >> 8) & 0xff); };
    auto u32 = [&](uint32_t v) { u16(v & 0xffff); u16(v >> 16); };
    u8('B'); u8('M'); u32(14 + 40 + row_bytes * (uint32_t)h); u16(0); u16(0); u32(14 + 40);   // file header
    u32(40); u32((uint32_t)w); u32((uint32_t)h); u16(1); u16(24);                            // bitmap header
    for (int k = 0; k < 6; ++k) u32(0);
    const unsigned char* px = (const unsigned char*)data;
    const int bg[3] = {255, 0, 255};
    for (int j = h - 1; j >= 0; --j) {
        for (int i = 0; i < w; ++i) {
            const unsigned char* d = px + ((size_t)j * w + i) * comp;
            if (comp <= 2) {
                u8(d[0]); u8(d[0]); u8(d[0]);
            } else if (comp == 3) {
                u8(d[2]); u8(d[1]); u8(d[0]);
            } else {
                unsigned char c[3];
                for (int k = 0; k < 3; ++k) c[k] = (unsigned char)(bg[k] + ((d[k] - bg[k]) * d[3]) / 255);
                u8(c[2]); u8(c[1]); u8(c[0]);
            }
        }
        for (int k = 0; k < pad; ++k) u8(0);
    }
    FILE* fp = fopen(path, "wb");
    if (!fp) return pt_internal_fail(PT_EINVAL, "cannot write %s", path);
    const size_t n = fwrite(f.data(), 1, f.size(), fp);
    const int closed = fclose(fp);
    if (n != f.size() || closed != 0) return pt_internal_fail(PT_EINVAL, "short write to %s", path);
    return PT_OK;
}

// LoadCubemapTexture (asset_loading.cpp:18-44): six faces loaded like LoadTexture (flipped), all
// assumed to share the LAST face's size (the reference reads Width/Height of the last file and
// copies faceSize floats from each); stacked vertically in file order (px nx py ny pz nz,
// Application.cpp:205-211).  Faces of a different size are an error here (the reference would
// read out of bounds).
int pt_load_cubemap_texture(const char* const paths[6], pt_texture* out)
{
    if (!paths || !out) return pt_internal_fail(PT_EINVAL, "null argument");
    memset(out, 0, sizeof(*out));
    pt_texture face[6] = {};
    int rc = PT_OK;
    for (int i = 0; i < 6 && rc == PT_OK; ++i) rc = pt_load_texture(paths[i], &face[i]);
    for (int i = 0; i < 6 && rc == PT_OK; ++i)
        if (face[i].width != face[5].width || face[i].height != face[5].height || face[i].components != 3)
            rc = pt_internal_fail(PT_EINVAL, "cubemap face %d is %dx%d, face 5 is %dx%d", i, face[i].width,
                                  face[i].height, face[5].width, face[5].height);
    if (rc == PT_OK) {
        const size_t fs = (size_t)face[5].width * face[5].height * 3;
        float* data = (float*)malloc(fs * 6 * sizeof(float));
        if (!data) {
            rc = pt_internal_fail(PT_ENOMEM, "out of host memory");
        } else {
            for (int i = 0; i < 6; ++i) memcpy(data + i * fs, face[i].data, fs * sizeof(float));
            out->data = data;
            out->width = face[5].width;
            out->height = face[5].height * 6;
            out->components = 3;
        }
    }
    for (int i = 0; i < 6; ++i) pt_free_texture(&face[i]);
    return rc;
}

void pt_free_texture(pt_texture* t)
{
    if (!t) return;
    free(t->data);
    memset(t, 0, sizeof(*t));
}

}  // extern "C"
