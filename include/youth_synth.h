/*
 * youth_synth.h — deterministic synthetic RGBD depth source.
 *
 * Stands in for the reference's SensorModule (Astra capture,
 * Youth.Source/SensorModule/sensorModule.c:69-264, astra_wrapper.cpp:38-52),
 * which needs hardware and an SDK absent here.  Produces the same buffer type
 * the sensor hands downstream: int16 [H][W] row-major depth in millimetres,
 * 0 = invalid (SLAM.h:22, viewerModule.c:341).
 *
 * Scene (SURVEY.md §8d "Synthetic inputs"): a 6 x 4 x 3 m room box, 8
 * spheres (r 0.3-0.55 m) on a ring and 3 oblique panels, ray-cast in fp64.
 * Depth = floor(Z*1000 + noise + 0.5) mm (noise sigma = 0.25 mm * Z^2, Z in m;
 * SURVEY §8d suggested 1.5 mm * Z^2, which leaves 1-px central-difference
 * normals unusable beyond ~2 m), kept only within 400..8000 mm,
 * ~2 % random holes.  RNG: SplitMix64.  Pair p of a batch uses seed
 * 0x5EED0000 + p; the 1000-frame sequence uses 0x5EED1000.
 *
 * Pure C, CPU only; no HIP.  Plain C-ABI.
 */
#ifndef YOUTH_SYNTH_H
#define YOUTH_SYNTH_H

#include <stdint.h>

#include "youth_icp.h"

#ifdef __cplusplus
extern "C" {
#endif

#define YOUTH_SYNTH_PAIR_SEED 0x5EED0000ull
#define YOUTH_SYNTH_SEQ_SEED  0x5EED1000ull

/* Flags for the generators. */
#define YOUTH_SYNTH_NOISE 1 /* add depth-dependent Gaussian noise (sigma = 0.25 mm * Z^2) */
#define YOUTH_SYNTH_HOLES 2 /* ~2 % random invalid pixels */
/* SURVEY §8d's optional noise level, sigma = 1.5 mm * Z^2 (replaces
 * YOUTH_SYNTH_NOISE's 0.25 when set): parity tests / bench leg only */
#define YOUTH_SYNTH_NOISE_SURVEY 4

/* Render one frame from the camera pose T_wc (4x4 row-major fp64; camera
 * frame x right, y down, z forward; world z up). */
void youth_synth_render(const double T_wc[16], int W, int H,
                        const youth_intrinsics* K, uint64_t noise_seed,
                        int flags, int16_t* depth);

/* One frame pair: random camera pose (seeded), small random motion
 * (rotation axis uniform on S^2, angle U(0, 1.5 deg), translation U(-15, 15)
 * mm per axis).  dst = frame at pose c0, src = frame at c1 = c0 * T_gt.
 * T_gt (nullable, 4x4 fp64) satisfies P_dst = T_gt * P_src — the quantity
 * ICP recovers. */
void youth_synth_pair(uint64_t seed, int W, int H, const youth_intrinsics* K,
                      int flags, int16_t* src, int16_t* dst, double* T_gt);

/* n pairs with seeds base_seed + first_index + p; src/dst [n][H][W]. */
void youth_synth_pairs(uint64_t base_seed, int first_index, int n, int W, int H,
                       const youth_intrinsics* K, int flags, int16_t* src,
                       int16_t* dst, double* T_gt);

/* Smooth trajectory (circle r = 1 m at ~1 cm/frame + yaw oscillation):
 * frames [n][H][W] and world poses T_wc [n][16] (nullable).  first_frame
 * lets a rank render only its shard [first_frame, first_frame + n). */
void youth_synth_sequence(uint64_t seed, int first_frame, int n, int W, int H,
                          const youth_intrinsics* K, int flags, int16_t* frames,
                          double* T_wc);

#ifdef __cplusplus
}
#endif

#endif
