/*
 * synth.c — deterministic synthetic depth source (see include/youth_synth.h).
 *
 * Replaces the Astra capture of the reference's SensorModule
 * (sensorModule.c:112, astra_wrapper.cpp:38-52) as the producer of int16 mm
 * depth frames.  Geometry is ray-cast in fp64; only the final quantisation
 * to int16 millimetres is shared with the consumer.  Built with
 * -ffp-contract=off so the same binary gives the same frames everywhere.
 */
#include "youth_synth.h"

#include <math.h>
#include <string.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* ---------------------------------------------------------------- RNG --- */
static uint64_t splitmix64(uint64_t* s)
{
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double u01(uint64_t* s) { return (double)(splitmix64(s) >> 11) * 0x1.0p-53; }
static double uniform(uint64_t* s, double lo, double hi) { return lo + (hi - lo) * u01(s); }

/* -------------------------------------------------------------- scene --- */
typedef struct { double c[3], r; } sphere_t;
typedef struct { double p0[3], e1[3], e2[3]; } panel_t;

static const double ROOM_MIN[3] = {-3.0, -2.0, 0.0};
static const double ROOM_MAX[3] = {3.0, 2.0, 3.0};

#define N_SPHERES 8
#define N_PANELS 3

static void scene_spheres(sphere_t sp[N_SPHERES])
{
    for (int k = 0; k < N_SPHERES; ++k) {
        const double a = (k * 45.0 + 10.0) * M_PI / 180.0;
        sp[k].c[0] = 2.2 * cos(a);
        sp[k].c[1] = 1.4 * sin(a);
        sp[k].c[2] = 0.5 + 0.3 * k;
        sp[k].r = 0.30 + 0.035 * k;
    }
}

static const panel_t PANELS[N_PANELS] = {
    {{2.2, -1.0, 0.0}, {0.0, 2.0, 0.0}, {0.7, 0.0, 2.2}},   /* ramp leaning on x=+3 */
    {{-1.5, -1.9, 0.8}, {1.2, 0.3, 0.0}, {0.2, 0.6, 1.0}},  /* tilted board near y=-2 */
    {{-2.8, 0.3, 0.7}, {0.0, 1.2, 0.0}, {0.9, 0.0, 0.4}},   /* slanted table near x=-3 */
};

static double dot3(const double a[3], const double b[3])
{
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}
static void cross3(const double a[3], const double b[3], double c[3])
{
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}
static void normalize3(double a[3])
{
    const double n = sqrt(dot3(a, a));
    a[0] /= n;
    a[1] /= n;
    a[2] /= n;
}

/* Nearest positive hit distance along o + t d (d not normalised). */
static double cast_ray(const double o[3], const double d[3], const sphere_t* sp)
{
    double t = INFINITY;
    for (int k = 0; k < 3; ++k) { /* room box from the inside */
        if (d[k] > 0.0) {
            const double tk = (ROOM_MAX[k] - o[k]) / d[k];
            if (tk < t) t = tk;
        } else if (d[k] < 0.0) {
            const double tk = (ROOM_MIN[k] - o[k]) / d[k];
            if (tk < t) t = tk;
        }
    }
    const double dd = dot3(d, d);
    for (int s = 0; s < N_SPHERES; ++s) {
        const double oc[3] = {o[0] - sp[s].c[0], o[1] - sp[s].c[1], o[2] - sp[s].c[2]};
        const double b = dot3(oc, d);
        const double c = dot3(oc, oc) - sp[s].r * sp[s].r;
        const double disc = b * b - dd * c;
        if (disc <= 0.0) continue;
        const double sq = sqrt(disc);
        double tk = (-b - sq) / dd;
        if (tk <= 1e-9) tk = (-b + sq) / dd;
        if (tk > 1e-9 && tk < t) t = tk;
    }
    for (int p = 0; p < N_PANELS; ++p) {
        const panel_t* P = &PANELS[p];
        double n[3];
        cross3(P->e1, P->e2, n);
        const double den = dot3(n, d);
        if (fabs(den) < 1e-12) continue;
        const double w[3] = {P->p0[0] - o[0], P->p0[1] - o[1], P->p0[2] - o[2]};
        const double tk = dot3(n, w) / den;
        if (!(tk > 1e-9 && tk < t)) continue;
        const double x[3] = {o[0] + tk * d[0] - P->p0[0], o[1] + tk * d[1] - P->p0[1],
                             o[2] + tk * d[2] - P->p0[2]};
        /* solve x = a e1 + b e2 in the panel plane (Gram system) */
        const double g11 = dot3(P->e1, P->e1), g12 = dot3(P->e1, P->e2),
                     g22 = dot3(P->e2, P->e2);
        const double r1 = dot3(x, P->e1), r2 = dot3(x, P->e2);
        const double det = g11 * g22 - g12 * g12;
        const double a = (r1 * g22 - r2 * g12) / det;
        const double bb = (r2 * g11 - r1 * g12) / det;
        if (a >= 0.0 && a <= 1.0 && bb >= 0.0 && bb <= 1.0) t = tk;
    }
    return t;
}

void youth_synth_render(const double T_wc[16], int W, int H,
                        const youth_intrinsics* K, uint64_t noise_seed,
                        int flags, int16_t* depth)
{
    sphere_t sp[N_SPHERES];
    scene_spheres(sp);
    const double o[3] = {T_wc[3], T_wc[7], T_wc[11]};
    uint64_t rng = noise_seed;
    for (int v = 0; v < H; ++v) {
        for (int u = 0; u < W; ++u) {
            /* camera ray with z-component 1, so the hit parameter is Z */
            const double dc[3] = {((double)u - K->cx) / K->fx, ((double)v - K->cy) / K->fy,
                                  1.0};
            double dw[3];
            for (int i = 0; i < 3; ++i)
                dw[i] = T_wc[i * 4 + 0] * dc[0] + T_wc[i * 4 + 1] * dc[1] +
                        T_wc[i * 4 + 2] * dc[2];
            const double z = cast_ray(o, dw, sp);
            /* always three draws per pixel, so flags do not shift the stream */
            const double hole = u01(&rng);
            const double g1 = (double)((splitmix64(&rng) >> 11) + 1) * 0x1.0p-53;
            const double g2 = u01(&rng);
            double zmm = z * (double)K->depth_scale;
            if (flags & (YOUTH_SYNTH_NOISE | YOUTH_SYNTH_NOISE_SURVEY)) {
                const double g = sqrt(-2.0 * log(g1)) * cos(2.0 * M_PI * g2);
                const double sigma = (flags & YOUTH_SYNTH_NOISE_SURVEY) ? 1.5 : 0.25;
                zmm += g * sigma * z * z * ((double)K->depth_scale / 1000.0);
            }
            double dq = floor(zmm + 0.5);
            const double lo = 0.4 * (double)K->depth_scale, hi = 8.0 * (double)K->depth_scale;
            if (!(dq >= lo && dq <= hi) || !isfinite(z)) dq = 0.0;
            if ((flags & YOUTH_SYNTH_HOLES) && hole < 0.02) dq = 0.0;
            if (dq > 32767.0) dq = 0.0;
            depth[(size_t)v * W + u] = (int16_t)dq;
        }
    }
}

/* T = [R t; 0 1] from camera orientation angles and position. */
static void camera_pose(double yaw, double pitch, double roll, const double pos[3],
                        double T[16])
{
    const double f[3] = {cos(pitch) * cos(yaw), cos(pitch) * sin(yaw), sin(pitch)};
    const double up[3] = {0.0, 0.0, 1.0};
    double r0[3], d0[3];
    cross3(f, up, r0);
    normalize3(r0);
    cross3(f, r0, d0);
    const double cr = cos(roll), sr = sin(roll);
    double r[3], d[3];
    for (int i = 0; i < 3; ++i) {
        r[i] = cr * r0[i] + sr * d0[i];
        d[i] = -sr * r0[i] + cr * d0[i];
    }
    for (int i = 0; i < 3; ++i) {
        T[i * 4 + 0] = r[i];
        T[i * 4 + 1] = d[i];
        T[i * 4 + 2] = f[i];
        T[i * 4 + 3] = pos[i];
    }
    T[12] = 0.0;
    T[13] = 0.0;
    T[14] = 0.0;
    T[15] = 1.0;
}

static void mat4_mul(const double A[16], const double B[16], double C[16])
{
    double O[16];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double s = 0.0;
            for (int k = 0; k < 4; ++k) s += A[i * 4 + k] * B[k * 4 + j];
            O[i * 4 + j] = s;
        }
    memcpy(C, O, sizeof(O));
}

void youth_synth_pair(uint64_t seed, int W, int H, const youth_intrinsics* K,
                      int flags, int16_t* src, int16_t* dst, double* T_gt)
{
    uint64_t s = seed;
    const double pos[3] = {uniform(&s, -0.3, 0.3), uniform(&s, -0.3, 0.3),
                           1.5 + uniform(&s, -0.3, 0.3)};
    const double yaw = uniform(&s, 0.0, 2.0 * M_PI);
    const double pitch = uniform(&s, -25.0, -5.0) * M_PI / 180.0;
    const double roll = uniform(&s, -8.0, 8.0) * M_PI / 180.0;
    double Twc0[16];
    camera_pose(yaw, pitch, roll, pos, Twc0);

    /* relative motion c0 -> c1: axis uniform on S^2, angle U(0, 1.5 deg) */
    double ax[3];
    do {
        for (int i = 0; i < 3; ++i) ax[i] = uniform(&s, -1.0, 1.0);
    } while (dot3(ax, ax) > 1.0 || dot3(ax, ax) < 1e-6);
    normalize3(ax);
    const double ang = uniform(&s, 0.0, 1.5) * M_PI / 180.0;
    const double c = cos(ang), sn = sin(ang), C = 1.0 - c;
    double T01[16] = {
        c + ax[0] * ax[0] * C, ax[0] * ax[1] * C - ax[2] * sn, ax[0] * ax[2] * C + ax[1] * sn, 0,
        ax[1] * ax[0] * C + ax[2] * sn, c + ax[1] * ax[1] * C, ax[1] * ax[2] * C - ax[0] * sn, 0,
        ax[2] * ax[0] * C - ax[1] * sn, ax[2] * ax[1] * C + ax[0] * sn, c + ax[2] * ax[2] * C, 0,
        0, 0, 0, 1};
    for (int i = 0; i < 3; ++i) T01[i * 4 + 3] = uniform(&s, -0.015, 0.015);
    double Twc1[16];
    mat4_mul(Twc0, T01, Twc1);
    const uint64_t seed_dst = splitmix64(&s);
    const uint64_t seed_src = splitmix64(&s);
    youth_synth_render(Twc0, W, H, K, seed_dst, flags, dst);
    youth_synth_render(Twc1, W, H, K, seed_src, flags, src);
    if (T_gt) memcpy(T_gt, T01, sizeof(T01));
}

void youth_synth_pairs(uint64_t base_seed, int first_index, int n, int W, int H,
                       const youth_intrinsics* K, int flags, int16_t* src,
                       int16_t* dst, double* T_gt)
{
    const size_t N = (size_t)W * (size_t)H;
    /* frames are independent (own seeds): parallel over pairs is deterministic */
#pragma omp parallel for schedule(dynamic, 1)
    for (int p = 0; p < n; ++p)
        youth_synth_pair(base_seed + (uint64_t)(first_index + p), W, H, K, flags,
                         src + (size_t)p * N, dst + (size_t)p * N,
                         T_gt ? T_gt + (size_t)p * 16 : NULL);
}

void youth_synth_sequence(uint64_t seed, int first_frame, int n, int W, int H,
                          const youth_intrinsics* K, int flags, int16_t* frames,
                          double* T_wc)
{
    const size_t N = (size_t)W * (size_t)H;
#pragma omp parallel for schedule(dynamic, 1)
    for (int f = 0; f < n; ++f) {
        const int k = first_frame + f;
        const double phi = 0.01 * k;
        const double pos[3] = {cos(phi), sin(phi), 1.5 + 0.05 * sin(0.03 * k)};
        const double yaw = phi + 0.35 * sin(0.02 * k);
        const double pitch = (-15.0 + 3.0 * sin(0.013 * k)) * M_PI / 180.0;
        const double roll = (2.0 * sin(0.017 * k)) * M_PI / 180.0;
        double T[16];
        camera_pose(yaw, pitch, roll, pos, T);
        uint64_t s = seed ^ (0xD1B54A32D192ED03ull * (uint64_t)(k + 1));
        const uint64_t ns = splitmix64(&s);
        youth_synth_render(T, W, H, K, ns, flags, frames + (size_t)f * N);
        if (T_wc) memcpy(T_wc + (size_t)f * 16, T, sizeof(T));
    }
}
