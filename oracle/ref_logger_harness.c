/*
 * ref_logger_harness.c — TEST INFRASTRUCTURE ONLY (never linked into the
 * product).  Drives the reference's own logger, compiled unchanged from
 * /root/reference/Youth.Source/LoggingModule/loggingModule.c (oracle/Makefile
 * target `ref`, output oracle/_ref/ref_logger), to produce golden fixtures
 * for SURVEY §8 f1/f2:
 *
 *   1. recording: frames are fed to the logger over MQ_SENSOR_TO_LOGGER in
 *      the sensor's message format (sensorModule.c:123-208: METADATA, depth
 *      chunks, colour chunks of MAX_MSG_SIZE - sizeof(MessageHeader) bytes);
 *      the logger reassembles them (loggingModule.c:291-357) and writes the
 *      .bin with its own saveFrameToFile (:101-130) and end marker
 *      (:224-226);
 *   2. playback: the logger's playback thread reads that file back
 *      (readFrameFromFile :404-444) and emits sendMetadata (:488-502) +
 *      sendDataInChunks (:447-485) on MQ_LOGGER_TO_VIEWER; every message is
 *      captured.
 *
 * Control goes through the reference's public API (startRecording,
 * sendControlCommand(CTRL_CMD_STOP_RECORD) — stopRecording() only sends when
 * NOT recording, loggingModule.c:703-707 — and startPlayback).  The logger
 * reads its control queue only after a sensor message arrives (:186 then
 * :278), so the harness follows each command with a marker METADATA message
 * (frameId kMarker) until the state flips; markers are dropped from the
 * capture.
 *
 * The reference leaves MessageHeader.ctrlCommand and .filename
 * (bytes 32..291) uninitialised in sendMetadata (stack) and sendDataInChunks
 * (malloc); the harness zeroes those bytes of every captured message, and the
 * tests compare them as zero.
 *
 * usage: ref_logger <frames.raw> <recording.bin> <playback.msgs>
 *   frames.raw:    u32 n; n x { u32 frameId, u32 timestamp, u32 W, u32 H,
 *                  int16 depth[W*H], u8 color[W*H*3] }
 *   playback.msgs: u32 count; count x { u32 len, len bytes }
 * The logger's threads are left running at exit (stopLoggingModule would
 * join a thread blocked in mq_receive, :682); the queues are unlinked.
 */
#define _GNU_SOURCE
#include <fcntl.h>
#include <mqueue.h>
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "LoggingModule/loggingModule.h"
#include "frameDefinitions.h"

enum { kMarker = 0x7F000001 };

typedef struct {
    uint32_t len;
    char* data;
} msg_t;

static msg_t* g_cap;
static size_t g_ncap, g_capcap;
static volatile int g_capture, g_drain_run = 1, g_drain_idle;
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;

static void sleep_ms(int ms)
{
    struct timespec ts = {ms / 1000, (long)(ms % 1000) * 1000000L};
    nanosleep(&ts, NULL);
}

static void* drain(void* arg)
{
    mqd_t q = *(mqd_t*)arg;
    char* buf = malloc(MAX_MSG_SIZE);
    while (g_drain_run) {
        struct timespec dl;
        clock_gettime(CLOCK_REALTIME, &dl);
        dl.tv_nsec += 20 * 1000000L;
        if (dl.tv_nsec >= 1000000000L) {
            dl.tv_sec += 1;
            dl.tv_nsec -= 1000000000L;
        }
        ssize_t n = mq_timedreceive(q, buf, MAX_MSG_SIZE, NULL, &dl);
        if (n <= 0) {
            g_drain_idle = 1;
            continue;
        }
        g_drain_idle = 0;
        const MessageHeader* h = (const MessageHeader*)buf;
        if (!g_capture || (n >= (ssize_t)sizeof(MessageHeader) && h->frameId == kMarker))
            continue;
        pthread_mutex_lock(&g_mu);
        if (g_ncap == g_capcap) {
            g_capcap = g_capcap ? 2 * g_capcap : 256;
            g_cap = realloc(g_cap, g_capcap * sizeof(msg_t));
        }
        char* m = malloc((size_t)n);
        memcpy(m, buf, (size_t)n);
        if (n >= (ssize_t)sizeof(MessageHeader))  /* uninitialised in the reference */
            memset(m + offsetof(MessageHeader, ctrlCommand), 0,
                   sizeof(MessageHeader) - offsetof(MessageHeader, ctrlCommand));
        g_cap[g_ncap].len = (uint32_t)n;
        g_cap[g_ncap].data = m;
        ++g_ncap;
        pthread_mutex_unlock(&g_mu);
    }
    free(buf);
    return NULL;
}

static void send_or_die(mqd_t q, const char* m, size_t n)
{
    if (mq_send(q, m, n, 0) != 0) {
        perror("mq_send");
        exit(3);
    }
}

/* sensorModule.c:123-135: the METADATA message */
static void send_meta(mqd_t q, char* buf, int fid, uint32_t ts, int W, int H)
{
    MessageHeader* h = (MessageHeader*)buf;
    memset(h, 0, sizeof(*h));
    h->msgType = MSG_TYPE_METADATA;
    h->width = W;
    h->height = H;
    h->chunkIndex = 0;
    h->totalChunks = 0;
    h->dataSize = 0;
    h->frameId = fid;
    h->timestamp = ts;
    send_or_die(q, buf, sizeof(MessageHeader));
}

/* sensorModule.c:137-208: one plane in MAX_MSG_SIZE - header chunks */
static void send_plane(mqd_t q, char* buf, int type, int fid, uint32_t ts, int W, int H,
                       const char* data, int size)
{
    const int per = MAX_MSG_SIZE - (int)sizeof(MessageHeader);
    const int total = (size + per - 1) / per;
    MessageHeader* h = (MessageHeader*)buf;
    for (int i = 0; i < total; ++i) {
        memset(h, 0, sizeof(*h));
        h->msgType = type;
        h->width = W;
        h->height = H;
        h->chunkIndex = i;
        h->totalChunks = total;
        h->frameId = fid;
        h->timestamp = ts;
        const int off = i * per;
        const int n = i == total - 1 ? size - off : per;
        h->dataSize = n;
        memcpy(buf + sizeof(MessageHeader), data + off, (size_t)n);
        send_or_die(q, buf, sizeof(MessageHeader) + (size_t)n);
    }
}

/* marker METADATA messages until cond() holds (the logger reads control
 * only after a sensor message, loggingModule.c:186,278) */
static int wait_state(mqd_t q, char* buf, int (*cond)(void))
{
    for (int k = 0; k < 500; ++k) {
        if (cond()) return 1;
        send_meta(q, buf, kMarker, 0, 8, 8);
        sleep_ms(10);
    }
    return cond();
}
static int is_rec(void) { return isRecording(); }
static int not_rec(void) { return !isRecording(); }
static int is_play(void) { return isPlayingBack(); }

int main(int argc, char** argv)
{
    if (argc != 4) {
        fprintf(stderr, "usage: %s frames.raw recording.bin playback.msgs\n", argv[0]);
        return 2;
    }
    FILE* fin = fopen(argv[1], "rb");
    uint32_t nf = 0;
    if (!fin || fread(&nf, 4, 1, fin) != 1) {
        perror("frames");
        return 2;
    }
    mq_unlink(MQ_SENSOR_TO_LOGGER);
    mq_unlink(MQ_LOGGER_TO_VIEWER);
    mq_unlink(MQ_CONTROL_QUEUE);
    remove(argv[2]);

    initLoggingModule();  /* creates the queues, starts logger + playback threads */
    mqd_t qs = mq_open(MQ_SENSOR_TO_LOGGER, O_WRONLY);
    mqd_t qv = mq_open(MQ_LOGGER_TO_VIEWER, O_RDONLY);
    if (qs == (mqd_t)-1 || qv == (mqd_t)-1) {
        perror("mq_open");
        return 3;
    }
    pthread_t dt;
    pthread_create(&dt, NULL, drain, &qv);
    char* buf = malloc(MAX_MSG_SIZE);

    if (!startRecording(argv[2]) || !wait_state(qs, buf, is_rec)) {
        fprintf(stderr, "recording did not start\n");
        return 4;
    }
    for (uint32_t k = 0; k < nf; ++k) {
        uint32_t hd[4];
        if (fread(hd, 4, 4, fin) != 4) return 2;
        const int W = (int)hd[2], H = (int)hd[3];
        const size_t dn = (size_t)W * H * 2, cn = (size_t)W * H * 3;
        char* d = malloc(dn + 1);
        char* c = malloc(cn + 1);
        if (fread(d, 1, dn, fin) != dn || fread(c, 1, cn, fin) != cn) return 2;
        send_meta(qs, buf, (int)hd[0], hd[1], W, H);
        send_plane(qs, buf, MSG_TYPE_DEPTH_DATA, (int)hd[0], hd[1], W, H, d, (int)dn);
        send_plane(qs, buf, MSG_TYPE_COLOR_DATA, (int)hd[0], hd[1], W, H, c, (int)cn);
        free(d);
        free(c);
    }
    fclose(fin);
    /* the logger reads control before each sensor message (:186, :278), and
     * up to mq_maxmsg frame messages may still be queued: stop only once the
     * sensor queue is empty (the last message's save then precedes the next
     * control read) */
    for (int k = 0; k < 1000; ++k) {
        struct mq_attr at;
        mq_getattr(qs, &at);
        if (at.mq_curmsgs == 0) break;
        sleep_ms(5);
    }
    sendControlCommand(CTRL_CMD_STOP_RECORD, NULL);
    if (!wait_state(qs, buf, not_rec)) {
        fprintf(stderr, "recording did not stop\n");
        return 4;
    }

    g_capture = 1;
    if (!startPlayback(argv[2]) || !wait_state(qs, buf, is_play)) {
        fprintf(stderr, "playback did not start\n");
        return 5;
    }
    for (int k = 0; k < 6000 && isPlayingBack(); ++k) sleep_ms(10);
    if (isPlayingBack()) {
        fprintf(stderr, "playback did not finish\n");
        return 5;
    }
    for (int k = 0; k < 500; ++k) {  /* queue empty and the drain idle */
        struct mq_attr at;
        mq_getattr(qv, &at);
        if (at.mq_curmsgs == 0 && g_drain_idle) break;
        sleep_ms(10);
    }
    g_drain_run = 0;
    pthread_join(dt, NULL);

    FILE* fo = fopen(argv[3], "wb");
    uint32_t cnt = (uint32_t)g_ncap;
    fwrite(&cnt, 4, 1, fo);
    for (size_t i = 0; i < g_ncap; ++i) {
        fwrite(&g_cap[i].len, 4, 1, fo);
        fwrite(g_cap[i].data, 1, g_cap[i].len, fo);
    }
    fclose(fo);
    mq_unlink(MQ_SENSOR_TO_LOGGER);
    mq_unlink(MQ_LOGGER_TO_VIEWER);
    mq_unlink(MQ_CONTROL_QUEUE);
    printf("ref_logger: %u frames recorded, %u playback messages\n", nf, cnt);
    fflush(stdout);
    _exit(0);
}
