/*
 * youth_viewer.h — C-ABI of the viewer's point list on MI355X.
 *
 * Replaces the data side of the reference viewer's 3-D view,
 * Youth.Source/ViewerModule/viewerModule.c:321-367 (display_3d_color):
 * that loop walks every pixel of the latest depth/colour frame on the CPU and
 * issues one glColor3f + glVertex3f per valid pixel (:336-357), 307,200
 * immediate-mode calls per 640x480 frame.  Here the same vertex list is built
 * on the GPU in one pass over HBM and handed out as a packed array a
 * renderer uploads as one vertex buffer (stride 24 B: glVertexPointer(3,
 * GL_FLOAT, 24, 0) + glColorPointer(3, GL_FLOAT, 24, 12)).  The GL side is
 * not part of this library (no GL headers in this build).
 *
 * Vertex k of a frame (raster order over the pixels with depth > 0, the loop
 * order of :336-339) is six floats {-x, -y, -z, r, g, b}, bit-identical to
 * the reference's glVertex3f / glColor3f arguments:
 *   z = d / 1000.0f; x = ((u - W/2) * z) / 570.3f; y = ((v - H/2) * z) / 570.3f
 *   (:343-345, with K = NULL; an explicit K generalises it exactly as the ICP
 *   back-projection does, youth_icp.h), r,g,b = rgb[3 index + c] / 255.0f
 *   (:349-352; rgb NULL gives colour 0).
 *
 * A context is used by one thread at a time; its device calls on one stream
 * run in order.  Plain C99, no HIP or torch types (streams travel as void*).  Entry points
 * return YOUTH_OK (0) / a count >= 0, or a negative YOUTH_E* code
 * (youth_icp.h); the text of the last error is youth_cloud_last_error().
 */
#ifndef YOUTH_VIEWER_H
#define YOUTH_VIEWER_H

#include <stddef.h>
#include <stdint.h>

#include "youth_icp.h"

#ifdef __cplusplus
extern "C" {
#endif

#define YOUTH_CLOUD_FLOATS_PER_VERTEX 6

typedef struct youth_cloud_ctx youth_cloud_ctx;

/* A builder for frames up to W x H (W, H <= 16384, W*H <= 2^26), up to
 * max_frames per device call, on HIP device `device`.  NULL on failure. */
youth_cloud_ctx* youth_cloud_create(int device, int W, int H, int max_frames);
void youth_cloud_destroy(youth_cloud_ctx* ctx);
const char* youth_cloud_last_error(void);

/* Device-resident batch of n_frames W x H frames (W, H <= the create size):
 *   d_depth    [n][H][W] int16, mm, 0 / negative = invalid (viewerModule.c:43,340)
 *   d_rgb      [n][H][W][3] uint8 RGB (viewerModule.c:44,348) or NULL
 *   d_vertices [n][W*H][6] float: frame f's list starts at f*W*H*6
 *   d_counts   [n] int32: vertices of frame f
 * Enqueued on `stream` (NULL: the context's stream); asynchronous. */
int youth_cloud_build_device(youth_cloud_ctx* ctx, const int16_t* d_depth,
                             const uint8_t* d_rgb, int n_frames, int W, int H,
                             const youth_intrinsics* K, float* d_vertices,
                             int32_t* d_counts, void* stream);

/* The same list in the WORLD frame, for a map view with the tracked poses
 * (the device point buffer plus the pose overlay): frame f's
 * camera-frame point P (the reference's x_pos, y_pos, z_pos) is moved by its
 * camera -> world pose, d_T_world[f] (device, fp32 row-major 3x4 [R | t]; the
 * first 12 entries of the SLAM trajectory's 4x4 T_w), as three fma chains
 *   X_w = fma(R02, z, fma(R01, y, fma(R00, x, t0)))   (likewise Y_w, Z_w),
 * the ICP transform's evaluation order, and the vertex is
 * {-X_w, -Y_w, -Z_w, r, g, b} (the reference's display flip, :354).
 * d_T_world NULL: exactly youth_cloud_build_device. */
int youth_cloud_build_device_posed(youth_cloud_ctx* ctx, const int16_t* d_depth,
                                   const uint8_t* d_rgb, int n_frames, int W, int H,
                                   const youth_intrinsics* K, const float* d_T_world,
                                   float* d_vertices, int32_t* d_counts, void* stream);

/* One host frame: copies depth (and rgb) in, builds, copies the list out.
 * vertices: room for `cap` vertices (cap >= W*H always suffices).  Returns
 * the vertex count (>= 0) or a negative YOUTH_E* code; synchronous. */
int youth_cloud_build_host(youth_cloud_ctx* ctx, const int16_t* depth, const uint8_t* rgb,
                           int W, int H, const youth_intrinsics* K, float* vertices,
                           int cap);

/* Wait for the work enqueued on `stream` (NULL: the context's stream). */
int youth_cloud_sync(youth_cloud_ctx* ctx, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* YOUTH_VIEWER_H */
