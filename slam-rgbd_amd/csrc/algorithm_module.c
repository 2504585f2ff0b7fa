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
 * has not already called initSlamModule), then runs the frame loop (SURVEY
 * §8b): it pulls the logger's frame messages from a 4th queue
 * (YOUTH_MQ_LOGGER_TO_ALGORITHM, or $YOUTH_ALGO_FRAME_QUEUE), reassembles
 * them, tracks each frame against the previous one and publishes the poses
 * on YOUTH_MQ_ALGORITHM_POSE ($YOUTH_ALGO_POSE_QUEUE; "" = none), until
 * stopSlamModule().  Callers may also hand frames in directly with
 * processSlamFrame (the logger's frame-complete point, loggingModule.c:354);
 * with YOUTH_ALGO_NO_QUEUE set, or if the queue cannot be opened, the thread
 * only parks until stopSlamModule().
 */
#include <stdio.h>
#include <stdlib.h>

#include "youth_icp.h"
#include "youth_wire.h"

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
    if (!getenv("YOUTH_ALGO_NO_QUEUE")) {
        const char* fq = getenv("YOUTH_ALGO_FRAME_QUEUE");
        const char* pq = getenv("YOUTH_ALGO_POSE_QUEUE");
        if (!fq || !*fq) fq = YOUTH_MQ_LOGGER_TO_ALGORITHM;
        if (!pq) pq = YOUTH_MQ_ALGORITHM_POSE;
        if (youth_algorithm_loop(fq, *pq ? pq : NULL, NULL) >= 0) return NULL;
        fprintf(stderr, "algorithmModule: frame queue unavailable; direct processSlamFrame only\n");
    }
    youth_slam_wait_stopped();
    return NULL;
}
