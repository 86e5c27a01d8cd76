/* Dev tool (not product, not the checker): per-(pixel, frame) path lengths of the scalar path, for
 * the tile-schedule simulator scripts/sim_schedule.py.  Reuses the oracle's restatement by
 * including it with one more instantiation whose CNT_SEG hook counts segments.
 * Build: gcc -O2 -ffp-contract=off -fPIC -shared -pthread scripts/sim_lengths.c -Ioracle -o build/libsimlen.so -lm */
#include "../oracle/pt_oracle.c"

static __thread unsigned g_len;
#undef SFX
#undef CNT
#undef CNTS
#undef CNT_T
#undef CNT_SEG
#undef CNT_ESC
#undef CNT_SAMP
#undef CNT_MARK
#undef CNT_PRIM
#undef CNT_SHARED
#undef CNT_SHARED_PRIM
#define SFX(n) n##_len
#define CNT(n) ((void)0)
#define CNTS(n) ((void)0)
#define CNT_T(n) ((void)0)
#define CNT_SEG() (g_len++)
#define CNT_ESC() ((void)0)
#define CNT_SAMP() ((void)0)
#define CNT_MARK() ((void)0)
#define CNT_PRIM() ((void)0)
#define CNT_SHARED(n) ((void)0)
#define CNT_SHARED_PRIM(d) ((void)0)
#include "../oracle/pt_oracle_core.inc"

typedef struct { const pto_params* p; uint8_t* out; int r0, r1; } sim_job;

static void* sim_rows(void* arg)
{
    sim_job* j = (sim_job*)arg;
    const pto_params* p = j->p;
    const float W = (float)p->width, H = (float)p->height, aspect = W / H;
    for (int gy = j->r0; gy < j->r1; ++gy) {
        const float fy = (float)(p->height - 1 - gy);
        for (int x = 0; x < p->width; ++x) {
            const float fx = (float)x;
            for (int f = 0; f < p->nframes; ++f) {
                const float iFrame = (float)(p->frame_first + (uint32_t)f);
                uint32_t rng = pto_seed((uint32_t)fx, (uint32_t)fy, (uint32_t)iFrame);
                float tx = (fx / W) * 2.0f - 1.0f, ty = (fy / H) * 2.0f - 1.0f;
                ty = ty / aspect;
                float t[3] = {tx - 0.0f, ty - 0.0f, g_cam_dist - 0.0f};
                float inv = 1.0f / sqrtf((t[0] * t[0] + t[1] * t[1]) + t[2] * t[2]);
                float D[3] = {t[0] * inv, t[1] * inv, t[2] * inv};
                const float P[3] = {0.0f, 0.0f, 0.0f};
                float c[3];
                g_len = 0;
                color_len(P, D, &rng, p, c);
                j->out[((size_t)gy * p->width + x) * p->nframes + f] = (uint8_t)g_len;
            }
        }
    }
    return 0;
}

/* out[(row * W + col) * nframes + f] = segments traced by sample (col, row, frame_first + f) */
int sim_lengths(int32_t w, int32_t h, uint32_t frame_first, int32_t nframes, int32_t bounces, uint8_t* out, int nthreads)
{
    pthread_once(&g_once, pto_init_scene);
    pto_params p;
    memset(&p, 0, sizeof(p));
    p.width = w; p.height = h; p.row_start = 0; p.row_stride = 1; p.nrows = h;
    p.frame_first = frame_first; p.nframes = nframes; p.num_bounces = bounces;
    p.ambient[0] = p.ambient[1] = p.ambient[2] = 0.1f;
    pthread_t th[64];
    sim_job jobs[64];
    if (nthreads > 64) nthreads = 64;
    for (int i = 0; i < nthreads; ++i) {
        jobs[i] = (sim_job){&p, out, (int)((int64_t)h * i / nthreads), (int)((int64_t)h * (i + 1) / nthreads)};
        pthread_create(&th[i], 0, sim_rows, &jobs[i]);
    }
    for (int i = 0; i < nthreads; ++i) pthread_join(th[i], 0);
    return 0;
}
