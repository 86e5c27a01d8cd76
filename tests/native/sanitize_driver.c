/* tests/native/sanitize_driver.c -- TEST INFRASTRUCTURE ONLY (tests/test_sanitizers.py).
 *
 * Runs the oracle restatements (oracle/pt_oracle.c: demofox_path_tracing_scalar.cpp incl. the config-4
 * env term; pt_oracle_output.c: the output stage; pt_oracle_v4.c: optimization_v4.cpp) on small
 * inputs, multi-threaded and counted, and writes every result to one binary file.  The test builds
 * this driver with the oracle sources under -fsanitize=address,undefined and
 * compares the file with the same results of the normal build (pyoracle) byte for byte: any
 * out-of-bounds access, use after free, leak or undefined arithmetic aborts the run, and the
 * sanitized build must not change a bit.
 *   sanitize_driver OUT.bin */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "pt_oracle.h"

static FILE* out;
static void put(const void* p, size_t n) { fwrite(p, 1, n, out); }

int main(int argc, char** argv)
{
    if (argc < 2) return 2;
    out = fopen(argv[1], "wb");
    if (!out) return 2;
    const int W = 48, H = 32;
    /* a small env map, deterministic (LCG), for config 4 and the v4 renderer */
    const int EW = 24, EH = 12;
    float* tex = malloc(sizeof(float) * EW * EH * 3);
    uint32_t lcg = 12345u;
    for (int i = 0; i < EW * EH * 3; ++i) {
        lcg = lcg * 1664525u + 1013904223u;
        tex[i] = 0.01f + (float)(lcg >> 8) * (3.0f / 16777216.0f);
    }
    pto_env env = {tex, EW, EH};
    /* scalar path: 8 bounces, 3 frames from frame 5, 4 threads, row shard 1::2 */
    float* buf = calloc((size_t)W * H * 3, sizeof(float));
    pto_params p = {W, H, 0, 1, H, 5, 3, 8, {0.1f, 0.1f, 0.1f}, NULL, 4};
    if (pto_render(buf, &p)) return 3;
    put(buf, sizeof(float) * W * H * 3);
    memset(buf, 0, sizeof(float) * W * H * 3);
    pto_params ps = {W, H, 1, 2, H / 2, 1, 2, 4, {0.1f, 0.1f, 0.1f}, &env, 3};
    if (pto_render(buf, &ps)) return 3;
    put(buf, sizeof(float) * W * (H / 2) * 3);
    /* counted (single thread) */
    memset(buf, 0, sizeof(float) * W * H * 3);
    pto_counts c;
    memset(&c, 0, sizeof(c));
    pto_params pc = {W, H, 0, 1, H, 1, 2, 8, {0.1f, 0.1f, 0.1f}, NULL, 1};
    if (pto_render_counted(buf, &pc, &c)) return 3;
    put(buf, sizeof(float) * W * H * 3);
    put(&c, sizeof(c));
    /* output stage, both formats, both non-default branches */
    uint32_t* px = malloc(sizeof(uint32_t) * W * H);
    pto_tonemap(buf, W, H, PTO_PIXEL_RGBA8, px);
    put(px, sizeof(uint32_t) * W * H);
    pto_tonemap_ex(buf, W, H, PTO_PIXEL_XRGB8, 1, 1, px);
    put(px, sizeof(uint32_t) * W * H);
    /* v4: default scene, equirect env, 2 frames, 2 threads; then the cubemap path (bilinear texels,
     * sin/cos unit vectors, exact exp) on six stacked 2x2 faces cut from the same texels */
    pto4_scene sc;
    pto4_default_scene(&sc);
    memset(buf, 0, sizeof(float) * W * H * 3);
    pto4_params p4 = {W, H, 0, 1, H, 1, 2, 8, PTO4_ENV_EQUIRECT, 1, 1, &env, 2, 0, 0};
    if (pto4_render(buf, &p4, &sc, NULL)) return 4;
    put(buf, sizeof(float) * W * H * 3);
    float cube[2 * 12 * 3];   /* 6 faces of 2x2 stacked: width 2, height 12 */
    for (int i = 0; i < 2 * 12 * 3; ++i) cube[i] = tex[i];
    pto_env cenv = {cube, 2, 12};
    memset(buf, 0, sizeof(float) * W * H * 3);
    pto4_params p4c = {W, H, 0, 1, H, 3, 2, 4, PTO4_ENV_CUBEMAP, 0, 0, &cenv, 1, 0, 1};
    pto4_counts c4;
    memset(&c4, 0, sizeof(c4));
    if (pto4_render(buf, &p4c, &sc, &c4)) return 4;
    put(buf, sizeof(float) * W * H * 3);
    put(&c4, sizeof(c4));
    free(px);
    free(buf);
    free(tex);
    fclose(out);
    return 0;
}
