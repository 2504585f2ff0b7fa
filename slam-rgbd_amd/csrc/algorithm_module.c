/*
 * algorithm_module.c — the AlgorithmModule thread entry, plain C99.
 *
 * Replaces Youth.Source/AlgorithmModule/algorithmModule.c:3-5, whose body
 * calls an undefined SLAM() (and whose header, SLAM.h:22, misses
 * <stdint.h>).  Signature unchanged (algorithmModule.h:6) so main.c's
 * commented-out launch (main.c:280-281)
 *
 *     pthread_t algorithm_thread_id;
 *     pthread_create(&algorithm_thread_id, NULL, algorithmModule, NULL);
 *
 * works as written.  The thread brings the HIP ICP module up (if the caller
 * has not already called initSlamModule) and parks until stopSlamModule();
 * frames arrive through processSlamFrame from the logger's frame-complete
 * point (loggingModule.c:354) on the caller's thread, exactly as SLAM.cpp's
 * queue + worker design intends.
 */
#include <stdio.h>
#include <stdlib.h>

#include "youth_icp.h"

void* algorithmModule(void* id)
{
    if (!isSlamModuleRunning()) {
        const char* cfg = (const char*)id;
        if (!cfg) cfg = getenv("YOUTH_SLAM_CONFIG");
        initSlamModule(cfg, NULL);
        if (!isSlamModuleRunning()) {
            fprintf(stderr, "algorithmModule: HIP ICP module failed to start\n");
            return NULL;
        }
    }
    youth_slam_wait_stopped();
    return NULL;
}
