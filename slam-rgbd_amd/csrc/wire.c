/*
 * wire.c — pipeline side of the drop-in (include/youth_wire.h; SURVEY §8
 * f1/f2), plain C99 like the reference's modules.
 *
 *   .bin recordings     writer as loggingModule.c:101-130 (saveFrameToFile)
 *                       + end marker :224-226; reader as :404-444
 *                       (readFrameFromFile), incl. its per-plane size cap
 *   chunked messages    sender as :447-500 (sendDataInChunks, sendMetadata),
 *                       reassembly as the logger's receive loop :299-354
 *   AlgorithmModule     a 4th queue carrying the same chunks; complete frames
 *                       go to processSlamFrame, new poses out as
 *                       YOUTH_MSG_TYPE_POSE messages
 */
#define _POSIX_C_SOURCE 200809L
#include "youth_wire.h"

#include <errno.h>
#include <fcntl.h>
#include <mqueue.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "youth_icp.h"

_Static_assert(sizeof(youth_frame_header) == 28, "FrameHeader is 28 B (frameDefinitions.h:11-20)");
_Static_assert(sizeof(youth_msg_header) == 292, "MessageHeader is 292 B (frameDefinitions.h:45-56)");
_Static_assert(YOUTH_MSG_PAYLOAD == 7900, "7900 payload bytes per chunk (loggingModule.c:455)");

#define REC_DEFAULT_CAP (1024u * 1024u) /* loggingModule.c:530 */
#define MAX_DIM 16384

/* ------------------------------------------------------------ recordings */

struct youth_rec_writer {
    FILE* f;
    int frames;
    int err;
};

youth_rec_writer* youth_rec_create(const char* path)
{
    if (!path) return NULL;
    youth_rec_writer* w = (youth_rec_writer*)calloc(1, sizeof(*w));
    if (!w) return NULL;
    w->f = fopen(path, "wb");
    if (!w->f) {
        free(w);
        return NULL;
    }
    return w;
}

static int write_zeros(FILE* f, size_t n)
{
    static const unsigned char z[4096];
    while (n) {
        const size_t k = n < sizeof(z) ? n : sizeof(z);
        if (fwrite(z, 1, k, f) != k) return 0;
        n -= k;
    }
    return 1;
}

int youth_rec_write_frame(youth_rec_writer* w, uint32_t frame_id, uint32_t timestamp_ms,
                          int width, int height, const int16_t* depth, const uint8_t* color)
{
    if (!w || !w->f || !depth || width <= 0 || height <= 0 || width > 65535 || height > 65535)
        return 0;
    const size_t n = (size_t)width * (size_t)height;
    if (n * 3 > 0xFFFFFFFFu) return 0;
    youth_frame_header h;
    memset(&h, 0, sizeof(h)); /* the 2 padding bytes too */
    h.frameId = frame_id;
    h.timestamp = timestamp_ms;
    h.frameType = YOUTH_FRAME_TYPE_DEPTH_COLOR;
    h.width = (uint16_t)width;
    h.height = (uint16_t)height;
    h.depthDataSize = (uint32_t)(n * sizeof(int16_t));
    h.colorDataSize = (uint32_t)(n * 3);
    int ok = fwrite(&h, sizeof(h), 1, w->f) == 1 &&
             fwrite(depth, sizeof(int16_t), n, w->f) == n &&
             (color ? fwrite(color, 1, n * 3, w->f) == n * 3 : write_zeros(w->f, n * 3)) &&
             fflush(w->f) == 0;
    if (!ok) {
        w->err = 1;
        return 0;
    }
    ++w->frames;
    return 1;
}

int youth_rec_close(youth_rec_writer* w)
{
    if (!w) return -1;
    int rc = w->err ? -1 : w->frames;
    if (w->f) {
        youth_frame_header end;
        memset(&end, 0, sizeof(end));
        end.frameType = YOUTH_FRAME_TYPE_END_OF_FILE;
        if (fwrite(&end, sizeof(end), 1, w->f) != 1) rc = -1;
        if (fclose(w->f) != 0) rc = -1;
    }
    free(w);
    return rc;
}

struct youth_rec_reader {
    FILE* f;
    uint32_t cap;
    int16_t* depth;
    size_t depth_bytes;
    uint8_t* color;
    size_t color_bytes;
};

youth_rec_reader* youth_rec_open(const char* path, uint32_t max_plane_bytes)
{
    if (!path) return NULL;
    youth_rec_reader* r = (youth_rec_reader*)calloc(1, sizeof(*r));
    if (!r) return NULL;
    r->f = fopen(path, "rb");
    if (!r->f) {
        free(r);
        return NULL;
    }
    r->cap = max_plane_bytes ? max_plane_bytes : REC_DEFAULT_CAP;
    return r;
}

static int grow(void** p, size_t* have, size_t need)
{
    if (need <= *have) return 1;
    void* q = realloc(*p, need);
    if (!q) return 0;
    *p = q;
    *have = need;
    return 1;
}

int youth_rec_next(youth_rec_reader* r, youth_frame_header* h, const int16_t** depth,
                   const uint8_t** color)
{
    if (!r || !r->f || !h) return -1;
    const size_t got = fread(h, 1, sizeof(*h), r->f);
    if (got == 0 && feof(r->f)) return 0; /* end of file without marker */
    if (got != sizeof(*h)) return -1;     /* truncated header */
    if (h->frameType == YOUTH_FRAME_TYPE_END_OF_FILE) return 0;
    if (h->depthDataSize > r->cap || h->colorDataSize > r->cap) return -1;
    const size_t n = (size_t)h->width * h->height;
    if (h->depthDataSize < n * sizeof(int16_t) || h->depthDataSize % sizeof(int16_t)) return -1;
    if (!grow((void**)&r->depth, &r->depth_bytes, h->depthDataSize ? h->depthDataSize : 2) ||
        !grow((void**)&r->color, &r->color_bytes, h->colorDataSize ? h->colorDataSize : 1))
        return -1;
    if (fread(r->depth, 1, h->depthDataSize, r->f) != h->depthDataSize) return -1;
    if (fread(r->color, 1, h->colorDataSize, r->f) != h->colorDataSize) return -1;
    if (depth) *depth = r->depth;
    if (color) *color = h->colorDataSize >= n * 3 ? r->color : NULL;
    return 1;
}

void youth_rec_close_reader(youth_rec_reader* r)
{
    if (!r) return;
    if (r->f) fclose(r->f);
    free(r->depth);
    free(r->color);
    free(r);
}

/* ------------------------------------------------------- chunked messages */

static int send_plane(youth_msg_sink sink, void* user, unsigned char* msg, int type,
                      uint32_t frame_id, uint32_t ts, int width, int height,
                      const unsigned char* data, int bytes)
{
    const int per = YOUTH_MSG_PAYLOAD;
    const int total = (bytes + per - 1) / per;
    for (int i = 0; i < total; ++i) {
        youth_msg_header h;
        memset(&h, 0, sizeof(h));
        h.msgType = type;
        h.width = width;
        h.height = height;
        h.chunkIndex = i;
        h.totalChunks = total;
        h.frameId = (int)frame_id;
        h.timestamp = ts;
        const int off = i * per;
        h.dataSize = i == total - 1 ? bytes - off : per;
        memcpy(msg, &h, sizeof(h));
        memcpy(msg + sizeof(h), data + off, (size_t)h.dataSize);
        if (sink(user, msg, sizeof(h) + (size_t)h.dataSize)) return -1;
    }
    return total;
}

int youth_wire_send_frame(youth_msg_sink sink, void* user, uint32_t frame_id,
                          uint32_t timestamp_ms, int width, int height, const int16_t* depth,
                          const uint8_t* color)
{
    if (!sink || !depth || width <= 0 || height <= 0 || width > MAX_DIM || height > MAX_DIM)
        return -1;
    unsigned char msg[YOUTH_MAX_MSG_SIZE];
    youth_msg_header h;
    memset(&h, 0, sizeof(h));
    h.msgType = YOUTH_MSG_TYPE_METADATA;
    h.width = width;
    h.height = height;
    h.frameId = (int)frame_id;
    h.timestamp = timestamp_ms;
    if (sink(user, &h, sizeof(h))) return -1;
    const int n = width * height;
    const int a = send_plane(sink, user, msg, YOUTH_MSG_TYPE_DEPTH_DATA, frame_id, timestamp_ms,
                             width, height, (const unsigned char*)depth, n * 2);
    if (a < 0) return -1;
    int b = 0;
    if (color) {
        b = send_plane(sink, user, msg, YOUTH_MSG_TYPE_COLOR_DATA, frame_id, timestamp_ms, width,
                       height, color, n * 3);
        if (b < 0) return -1;
    }
    return 1 + a + b;
}

struct youth_frame_asm {
    int need_color;
    int width, height;
    int16_t* depth;
    size_t depth_bytes;
    uint8_t* color;
    size_t color_bytes;
    int got_depth, got_color;
    int frame_id;
    uint32_t ts;
};

youth_frame_asm* youth_asm_create(int need_color)
{
    youth_frame_asm* a = (youth_frame_asm*)calloc(1, sizeof(*a));
    if (a) a->need_color = need_color;
    return a;
}

void youth_asm_destroy(youth_frame_asm* a)
{
    if (!a) return;
    free(a->depth);
    free(a->color);
    free(a);
}

int youth_asm_push(youth_frame_asm* a, const void* msg, size_t len, youth_frame_header* out,
                   const int16_t** depth, const uint8_t** color)
{
    if (!a || !msg || len < sizeof(youth_msg_header)) return -1;
    youth_msg_header h;
    memcpy(&h, msg, sizeof(h));
    const unsigned char* payload = (const unsigned char*)msg + sizeof(h);
    switch (h.msgType) {
    case YOUTH_MSG_TYPE_METADATA: /* reallocateBuffers, loggingModule.c:301-310 */
        if (h.width <= 0 || h.height <= 0 || h.width > MAX_DIM || h.height > MAX_DIM) return -1;
        {
            const size_t n = (size_t)h.width * h.height;
            if (!grow((void**)&a->depth, &a->depth_bytes, n * 2) ||
                !grow((void**)&a->color, &a->color_bytes, n * 3))
                return -1;
        }
        a->width = h.width;
        a->height = h.height;
        a->got_depth = a->got_color = 0;
        a->frame_id = h.frameId;
        a->ts = h.timestamp;
        return 0;
    case YOUTH_MSG_TYPE_DEPTH_DATA:
    case YOUTH_MSG_TYPE_COLOR_DATA: { /* :312-350 */
        const int is_depth = h.msgType == YOUTH_MSG_TYPE_DEPTH_DATA;
        if (h.dataSize < 0 || h.dataSize > YOUTH_MSG_PAYLOAD || h.chunkIndex < 0 ||
            len < sizeof(h) + (size_t)h.dataSize)
            return -1;
        int* got = is_depth ? &a->got_depth : &a->got_color;
        if (h.chunkIndex == 0) *got = 0;
        unsigned char* plane = is_depth ? (unsigned char*)a->depth : a->color;
        const size_t plane_bytes =
            (size_t)a->width * a->height * (is_depth ? 2 : 3); /* current frame size */
        if (plane) {
            const size_t off = (size_t)h.chunkIndex * YOUTH_MSG_PAYLOAD;
            if (off + (size_t)h.dataSize <= plane_bytes) memcpy(plane + off, payload, h.dataSize);
            if (h.chunkIndex == h.totalChunks - 1) *got = 1;
        }
        a->frame_id = h.frameId;
        a->ts = h.timestamp;
        break;
    }
    default:
        return 0; /* control and other types are not frame data */
    }
    if (!a->got_depth || (a->need_color && !a->got_color)) return 0;
    if (out) {
        memset(out, 0, sizeof(*out));
        out->frameId = (uint32_t)a->frame_id;
        out->timestamp = a->ts;
        out->frameType = YOUTH_FRAME_TYPE_DEPTH_COLOR;
        out->width = (uint16_t)a->width;
        out->height = (uint16_t)a->height;
        out->depthDataSize = (uint32_t)((size_t)a->width * a->height * 2);
        out->colorDataSize = a->got_color ? (uint32_t)((size_t)a->width * a->height * 3) : 0;
    }
    if (depth) *depth = a->depth;
    if (color) *color = a->got_color ? a->color : NULL;
    a->got_depth = a->got_color = 0; /* report each frame once */
    return 1;
}

/* ------------------------------------------------- AlgorithmModule loop */

#define TS_RING 64

static void deadline_in(struct timespec* t, long ms)
{
    clock_gettime(CLOCK_REALTIME, t);
    t->tv_nsec += ms * 1000000L;
    while (t->tv_nsec >= 1000000000L) {
        t->tv_nsec -= 1000000000L;
        ++t->tv_sec;
    }
}

static mqd_t open_queue(const char* name, int flags)
{
    struct mq_attr attr;
    memset(&attr, 0, sizeof(attr));
    attr.mq_maxmsg = YOUTH_MQ_MAXMSG;
    attr.mq_msgsize = YOUTH_MAX_MSG_SIZE;
    return mq_open(name, flags | O_CREAT, 0644, &attr);
}

static int mq_sink(void* user, const void* msg, size_t len)
{
    return mq_send(*(mqd_t*)user, (const char*)msg, len, 0) == -1;
}

int youth_algorithm_run(youth_msg_source recv, void* recv_user, youth_msg_sink publish,
                        void* publish_user, volatile int* stop)
{
    if (!recv) return -1;
    youth_frame_asm* as = youth_asm_create(0);
    unsigned char* buf = (unsigned char*)malloc(YOUTH_MAX_MSG_SIZE);
    if (!as || !buf) {
        youth_asm_destroy(as);
        free(buf);
        return -1;
    }
    uint32_t ring_ts[TS_RING];
    int ring_id[TS_RING];
    int ring_n = 0, frames = 0, published = 0;
    /* *stop is written by another thread: read it atomically (the writer
     * should store atomically too, youth_wire.h) */
    while (!(stop && __atomic_load_n(stop, __ATOMIC_ACQUIRE)) && isSlamModuleRunning()) {
        const int n = recv(recv_user, buf, YOUTH_MAX_MSG_SIZE, 50);
        if (n < 0) break;
        if (n > 0) {
            youth_frame_header h;
            const int16_t* d = NULL;
            const uint8_t* c = NULL;
            if (youth_asm_push(as, buf, (size_t)n, &h, &d, &c) == 1 &&
                processSlamFrame(d, c, h.width, h.height, h.timestamp) == 1) {
                ring_ts[ring_n % TS_RING] = h.timestamp;
                ring_id[ring_n % TS_RING] = (int)h.frameId;
                ++ring_n;
                ++frames;
            }
        }
        if (!publish) continue;
        const int len = youth_slam_trajectory_length();
        if (len < published) published = 0; /* a new sequence restarted the trajectory */
        while (published < len) {
            unsigned char msg[sizeof(youth_msg_header) + sizeof(youth_pose_msg)];
            youth_msg_header h;
            youth_pose_msg p;
            memset(&h, 0, sizeof(h));
            memset(&p, 0, sizeof(p));
            uint32_t ts = 0;
            if (youth_slam_get_pose(published, &ts, p.T_wc) != 1) break;
            p.index = published;
            h.msgType = YOUTH_MSG_TYPE_POSE;
            h.dataSize = (int)sizeof(p);
            h.timestamp = ts;
            h.frameId = -1; /* the frame this pose belongs to, matched by timestamp */
            for (int k = ring_n - 1; k >= 0 && k >= ring_n - TS_RING; --k)
                if (ring_ts[k % TS_RING] == ts) {
                    h.frameId = ring_id[k % TS_RING];
                    break;
                }
            memcpy(msg, &h, sizeof(h));
            memcpy(msg + sizeof(h), &p, sizeof(p));
            publish(publish_user, msg, sizeof(msg));
            ++published;
        }
    }
    free(buf);
    youth_asm_destroy(as);
    return frames;
}

static int mq_source(void* user, void* buf, size_t cap, int timeout_ms)
{
    struct timespec dl;
    deadline_in(&dl, timeout_ms);
    const ssize_t n = mq_timedreceive(*(mqd_t*)user, (char*)buf, cap, NULL, &dl);
    if (n >= 0) return (int)n;
    return errno == ETIMEDOUT || errno == EINTR ? 0 : -1;
}

static int mq_pose_sink(void* user, const void* msg, size_t len)
{
    /* non-blocking queue: a full pose queue drops the message */
    if (mq_send(*(mqd_t*)user, (const char*)msg, len, 0) == -1 && errno != EAGAIN)
        perror("youth_algorithm_loop: mq_send pose");
    return 0;
}

int youth_algorithm_loop(const char* frame_queue, const char* pose_queue, volatile int* stop)
{
    if (!frame_queue) return -1;
    mqd_t in = open_queue(frame_queue, O_RDONLY); /* attrs: loggingModule.c:138-141 */
    if (in == (mqd_t)-1) {
        perror("youth_algorithm_loop: mq_open frame queue");
        return -1;
    }
    mqd_t out = (mqd_t)-1;
    if (pose_queue) {
        out = open_queue(pose_queue, O_WRONLY | O_NONBLOCK);
        if (out == (mqd_t)-1) {
            perror("youth_algorithm_loop: mq_open pose queue");
            mq_close(in);
            return -1;
        }
    }
    const int frames = youth_algorithm_run(mq_source, &in, out != (mqd_t)-1 ? mq_pose_sink : NULL,
                                           &out, stop);
    mq_close(in);
    if (out != (mqd_t)-1) mq_close(out);
    return frames;
}

int youth_wire_mq_send_frame(const char* queue, uint32_t frame_id, uint32_t timestamp_ms,
                             int width, int height, const int16_t* depth, const uint8_t* color)
{
    if (!queue) return -1;
    mqd_t q = open_queue(queue, O_WRONLY);
    if (q == (mqd_t)-1) return -1;
    const int n = youth_wire_send_frame(mq_sink, &q, frame_id, timestamp_ms, width, height, depth,
                                        color);
    mq_close(q);
    return n;
}

int youth_wire_mq_recv_pose(const char* queue, int timeout_ms, youth_msg_header* h,
                            youth_pose_msg* pose)
{
    if (!queue) return -1;
    mqd_t q = open_queue(queue, O_RDONLY);
    if (q == (mqd_t)-1) return -1;
    unsigned char buf[YOUTH_MAX_MSG_SIZE];
    int rc = -1;
    for (;;) {
        ssize_t n;
        if (timeout_ms < 0) {
            n = mq_receive(q, (char*)buf, sizeof(buf), NULL);
        } else {
            struct timespec dl;
            deadline_in(&dl, timeout_ms);
            n = mq_timedreceive(q, (char*)buf, sizeof(buf), NULL, &dl);
        }
        if (n < 0) {
            rc = errno == ETIMEDOUT ? 0 : -1;
            break;
        }
        youth_msg_header mh;
        if ((size_t)n < sizeof(mh)) continue;
        memcpy(&mh, buf, sizeof(mh));
        if (mh.msgType != YOUTH_MSG_TYPE_POSE || mh.dataSize != (int)sizeof(youth_pose_msg) ||
            (size_t)n < sizeof(mh) + sizeof(youth_pose_msg))
            continue; /* not a pose: skip */
        if (h) *h = mh;
        if (pose) memcpy(pose, buf + sizeof(mh), sizeof(*pose));
        rc = 1;
        break;
    }
    mq_close(q);
    return rc;
}

int youth_rec_play(const char* path, int realtime)
{
    youth_rec_reader* r = youth_rec_open(path, 0xFFFFFFFFu); /* own playback: no 1 MiB cap */
    if (!r) return -1;
    int frames = 0, rc;
    youth_frame_header h;
    const int16_t* d;
    const uint8_t* c;
    while ((rc = youth_rec_next(r, &h, &d, &c)) == 1) {
        if (processSlamFrame(d, c, h.width, h.height, h.timestamp) != 1) {
            rc = -1;
            break;
        }
        ++frames;
        if (realtime) {
            struct timespec t = {0, 33333000L}; /* loggingModule.c:599 */
            nanosleep(&t, NULL);
        } else {
            youth_slam_wait_idle(60000); /* no drops: the queue never overflows */
        }
    }
    youth_rec_close_reader(r);
    return rc < 0 ? -1 : frames;
}
