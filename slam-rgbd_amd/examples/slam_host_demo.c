/*
 * slam_host_demo.c — plain-C99 host driving the drop-in exactly the way the
 * reference's process would (Youth.Source/main.c:279-281 launches the
 * algorithm thread; the logger's frame-complete point loggingModule.c:354
 * hands over each reassembled frame):
 *
 *   pthread_create(&tid, NULL, algorithmModule, config)   // main.c:280-281
 *   processSlamFrame(depth, color, w, h, ts)              // per frame
 *   saveSlamMap(base)                                      // SLAM.h:27
 *   stopSlamModule(); pthread_join(tid)
 *
 * Frames come from the synthetic depth source (stand-in for the Astra
 * SensorModule).  Prints one line per tracked frame and exits 0 when every
 * frame was tracked and the TUM file was written.
 *
 * usage: slam_host_demo <config.yaml|-> <n_frames> <out_base>
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "youth_icp.h"
#include "youth_synth.h"

int main(int argc, char** argv)
{
    const char* cfg = argc > 1 && strcmp(argv[1], "-") != 0 ? argv[1] : NULL;
    const int n = argc > 2 ? atoi(argv[2]) : 10;
    const char* base = argc > 3 ? argv[3] : "/tmp/youth_demo";
    const int W = 640, H = 480;
    youth_intrinsics K = youth_default_intrinsics(W, H);

    pthread_t tid;
    if (pthread_create(&tid, NULL, algorithmModule, (void*)cfg) != 0) return 2;
    for (int i = 0; i < 500 && !isSlamModuleRunning(); ++i) {
        struct timespec ts = {0, 10 * 1000 * 1000};
        nanosleep(&ts, NULL);
    }
    if (!isSlamModuleRunning()) {
        fprintf(stderr, "demo: module did not start\n");
        pthread_join(tid, NULL);
        return 3;
    }
    int16_t* frame = (int16_t*)malloc((size_t)W * H * sizeof(int16_t));
    uint8_t* color = (uint8_t*)calloc((size_t)W * H * 3, 1);
    for (int k = 0; k < n; ++k) {
        youth_synth_sequence(YOUTH_SYNTH_SEQ_SEED, k, 1, W, H, &K,
                             YOUTH_SYNTH_NOISE | YOUTH_SYNTH_HOLES, frame, NULL);
        if (processSlamFrame(frame, color, W, H, (uint32_t)(33 * k)) != 1) return 4;
        youth_slam_wait_idle(20000); /* a live sensor paces at 33 ms (sensorModule.c:243) */
        printf("frame %d tracked, map points %d\n", k, getSlamMapPoints());
    }
    const int traj = youth_slam_trajectory_length();
    const int saved = saveSlamMap(base);
    stopSlamModule();
    pthread_join(tid, NULL);
    free(frame);
    free(color);
    printf("trajectory %d poses, saved=%d (%s_trajectory.txt)\n", traj, saved, base);
    return (traj == n && saved == 1) ? 0 : 5;
}
