/* include/pt_flags.h -- bridge from the reference's compile-time configuration to the runtime one.
 *
 * A host that keeps the reference's global_preprocessor_flags.h (CPUPerformanceRayTracer/
 * global_preprocessor_flags.h) includes it, then this header, and calls
 * pt_apply_global_preprocessor_flags() once before rendering (e.g. next to
 * InitializeGlobalRenderResources, Application.cpp:413).  Whichever of the reference's macros the
 * host defines are applied through pt_init (pt_config) and pt_v4_set_config (pt_v4_config); macros
 * it does not define keep the reference's defaults.  Renderer macros read:
 *
 *   NUM_SAMPLES_PER_FRAME (flags.h:30/33)    pt_config.samples_per_frame (frame calls of the
 *                                            diffuse path accumulate that many frames)
 *   USE_ENV_MAP, USE_ENV_CUBEMAP (:56-57)    pt_v4_config.env_mode
 *   OUTPUT_TO_SCREEN (:58)                   pt_v4_config.output_to_screen
 *   ACCUMULATE_FRAMES (:60)                  pt_v4_config.accumulate_frames
 *   USE_FAST_APPROXIMATE_GAMMA (:62)         pt_v4_config.fast_gamma
 *   USE_FAST_APPROXIMATE_ACES_TONEMAP (:63)  pt_v4_config.fast_aces
 *   USE_FAST_APPROXIMATE_EXP (:64)           pt_v4_config.fast_exp
 *   USE_UNIT_VECTOR_REJECTION_SAMPLING (:65) pt_v4_config.rejection
 *   USE_RANDOM_JITTER_TEXTURE_SAMPLING (:66) pt_v4_config.random_jitter
 * plus this backend's own optional macros: PT_NUM_BOUNCES (the diffuse path's c_numBounces,
 * demofox_path_tracing_scalar.cpp:19, a file constant in the reference), PT_V4_NUM_BOUNCES
 * (c_numBounces, v4 :23) and PT_DEVICES (a string such as "0,1,2,3" or "all": the GPUs frames are
 * dealt to; default: the PT_MI355_DEVICES environment variable, else device 0).
 *
 * Not applicable on the GPU (accepted, no effect): USE_NON_TEMPORAL_STORE (:59, the accumulator is
 * read and written once per launch), NUM_THREADS (:69, the GPU grid replaces the CPU workers),
 * NUM_TILES_X / NUM_TILES_Y and RENDER_BUFFER_PIXEL_* (the host passes them to every call),
 * VISUALIZE_TILES (:72, colours tiles by CPU thread id -- nondeterministic in the reference).
 *
 * Returns PT_OK or the failing call's PT_E* code.  It (re)initialises the backend (pt_init resets
 * the frame counters, like a fresh process of the reference).
 */
#ifndef PT_FLAGS_H
#define PT_FLAGS_H
#include <stdlib.h>
#include "pt_mi355.h"

#ifdef __cplusplus
extern "C" {
#endif

static inline int pt_apply_global_preprocessor_flags(void)
{
    pt_config c;
    pt_v4_config v;
    int rc;
    pt_default_config(&c);   /* also reads PT_MI355_DEVICES */
#ifdef PT_DEVICES
    setenv("PT_MI355_DEVICES", PT_DEVICES, 1);   /* parsed by pt_default_config ("all" or ordinals) */
    pt_default_config(&c);
#endif
#ifdef NUM_SAMPLES_PER_FRAME
    c.samples_per_frame = NUM_SAMPLES_PER_FRAME;
#endif
#ifdef PT_NUM_BOUNCES
    c.num_bounces = PT_NUM_BOUNCES;
#endif
    if ((rc = pt_init(&c)) != PT_OK) return rc;

    pt_v4_default_config(&v);
#ifdef USE_ENV_MAP
#if USE_ENV_MAP
#if defined(USE_ENV_CUBEMAP) && USE_ENV_CUBEMAP
    v.env_mode = PT_V4_ENV_CUBEMAP;
#else
    v.env_mode = PT_V4_ENV_EQUIRECT;
#endif
#else
    v.env_mode = PT_V4_ENV_NONE;
#endif
#endif
#ifdef OUTPUT_TO_SCREEN
    v.output_to_screen = (OUTPUT_TO_SCREEN) ? 1 : 0;
#endif
#ifdef ACCUMULATE_FRAMES
    v.accumulate_frames = (ACCUMULATE_FRAMES) ? 1 : 0;
#endif
#ifdef USE_FAST_APPROXIMATE_GAMMA
    v.fast_gamma = (USE_FAST_APPROXIMATE_GAMMA) ? 1 : 0;
#endif
#ifdef USE_FAST_APPROXIMATE_ACES_TONEMAP
    v.fast_aces = (USE_FAST_APPROXIMATE_ACES_TONEMAP) ? 1 : 0;
#endif
#ifdef USE_FAST_APPROXIMATE_EXP
    v.fast_exp = (USE_FAST_APPROXIMATE_EXP) ? 1 : 0;
#endif
#ifdef USE_UNIT_VECTOR_REJECTION_SAMPLING
    v.rejection = (USE_UNIT_VECTOR_REJECTION_SAMPLING) ? 1 : 0;
#endif
#ifdef USE_RANDOM_JITTER_TEXTURE_SAMPLING
    v.random_jitter = (USE_RANDOM_JITTER_TEXTURE_SAMPLING) ? 1 : 0;
#endif
#ifdef PT_V4_NUM_BOUNCES
    v.num_bounces = PT_V4_NUM_BOUNCES;
#endif
    return pt_v4_set_config(&v);
}

#ifdef __cplusplus
}
#endif
#endif
