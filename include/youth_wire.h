/*
 * youth_wire.h — the pipeline side of the drop-in: the
 * Sensor -> Logging -> Algorithm wire formats, the `.bin` recording format,
 * and the AlgorithmModule frame loop.  Plain C99, no HIP types.
 *
 * The first part MIRRORS Youth.Source/frameDefinitions.h (layouts, values
 * and sizes unchanged, checked by static asserts here and by
 * tests/test_abi.py) so the library can speak to the reference's modules
 * without including their header.  The second part is ADDITIVE only: new
 * defines in this separate header (SURVEY §8b "Wire contract upstream"); no
 * existing layout changes.
 */
#ifndef YOUTH_WIRE_H
#define YOUTH_WIRE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- mirror of frameDefinitions.h -------------------------------------- */

#define YOUTH_FRAME_TYPE_DEPTH_COLOR 1    /* frameDefinitions.h:7 */
#define YOUTH_FRAME_TYPE_END_OF_FILE 0xFF /* frameDefinitions.h:8 */

/* FrameHeader (frameDefinitions.h:11-20): one per recorded frame, 28 B. */
typedef struct youth_frame_header {
    uint32_t frameId;
    uint32_t timestamp;     /* ms */
    uint16_t frameType;     /* YOUTH_FRAME_TYPE_* */
    uint16_t width;
    uint16_t height;
    uint32_t depthDataSize; /* bytes: W*H*2 */
    uint32_t colorDataSize; /* bytes: W*H*3 */
    uint32_t reserved;
} youth_frame_header;

#define YOUTH_MSG_TYPE_METADATA   1 /* frameDefinitions.h:33 */
#define YOUTH_MSG_TYPE_DEPTH_DATA 2 /* :34 */
#define YOUTH_MSG_TYPE_COLOR_DATA 3 /* :35 */
#define YOUTH_MSG_TYPE_CONTROL    4 /* :36 */

#define YOUTH_CTRL_CMD_START_RECORD   1 /* :39-42 */
#define YOUTH_CTRL_CMD_STOP_RECORD    2
#define YOUTH_CTRL_CMD_START_PLAYBACK 3
#define YOUTH_CTRL_CMD_STOP_PLAYBACK  4

/* MessageHeader (frameDefinitions.h:45-56): every mq message starts with
 * one, 292 B; the payload follows it in the same message. */
typedef struct youth_msg_header {
    int msgType;
    int width;
    int height;
    int chunkIndex;
    int totalChunks;
    int dataSize; /* payload bytes in this message */
    int frameId;
    uint32_t timestamp;
    int ctrlCommand;
    char filename[256];
} youth_msg_header;

#define YOUTH_MQ_SENSOR_TO_LOGGER "/sensor_logger_queue" /* :59 */
#define YOUTH_MQ_LOGGER_TO_VIEWER "/logger_viewer_queue" /* :60 */
#define YOUTH_MQ_CONTROL_QUEUE    "/control_queue"       /* :61 */
#define YOUTH_MAX_MSG_SIZE        8192                   /* :64 */
/* payload bytes per chunk message (loggingModule.c:455): 7900 */
#define YOUTH_MSG_PAYLOAD (YOUTH_MAX_MSG_SIZE - (int)sizeof(youth_msg_header))
/* mq depth the reference opens its queues with (loggingModule.c:139) */
#define YOUTH_MQ_MAXMSG 10

/* ---- additions (new defines only) --------------------------------------- */

/* A 4th queue carrying the logger's frame messages to the AlgorithmModule
 * (the same 292-B-header chunks it forwards to the viewer), and a queue the
 * AlgorithmModule publishes poses on. */
#define YOUTH_MQ_LOGGER_TO_ALGORITHM "/logger_algorithm_queue"
#define YOUTH_MQ_ALGORITHM_POSE      "/algorithm_pose_queue"

/* A pose message is a youth_msg_header with msgType = YOUTH_MSG_TYPE_POSE,
 * frameId/timestamp of the tracked frame, dataSize = sizeof(youth_pose_msg),
 * followed by this payload. */
#define YOUTH_MSG_TYPE_POSE 5
typedef struct youth_pose_msg {
    int32_t index;     /* position in the trajectory (0 = world origin) */
    int32_t reserved;
    double T_wc[16];   /* world <- camera, row-major 4x4, fp64 */
} youth_pose_msg;

/* ---- .bin recordings (loggingModule.c:101-130 writer, :404-444 reader) --- */

typedef struct youth_rec_writer youth_rec_writer;
typedef struct youth_rec_reader youth_rec_reader;

/* Create/truncate a recording.  NULL on failure. */
youth_rec_writer* youth_rec_create(const char* path);
/* Append one frame: FrameHeader (frameType DEPTH_COLOR) + W*H int16 depth +
 * W*H*3 uint8 colour (color may be NULL: zeros are written, keeping the
 * layout).  Flushed per frame, as the logger does.  1 on success, 0 on error. */
int youth_rec_write_frame(youth_rec_writer* w, uint32_t frame_id, uint32_t timestamp_ms,
                          int width, int height, const int16_t* depth, const uint8_t* color);
/* Write the end-of-file marker (a zero FrameHeader with frameType 0xFF,
 * loggingModule.c:224-226) and close.  Returns the number of frames written,
 * or -1 on an I/O error. */
int youth_rec_close(youth_rec_writer* w);

/* Open a recording for reading; planes larger than max_plane_bytes are
 * rejected as the logger's playback does (0 selects its 1 MiB cap,
 * loggingModule.c:530).  NULL on failure. */
youth_rec_reader* youth_rec_open(const char* path, uint32_t max_plane_bytes);
/* Next frame: 1 and *h, *depth, *color filled (pointers into reader-owned
 * buffers, valid until the next call); 0 at the end marker or end of file;
 * -1 on a truncated frame or a plane over the cap. */
int youth_rec_next(youth_rec_reader* r, youth_frame_header* h, const int16_t** depth,
                   const uint8_t** color);
void youth_rec_close_reader(youth_rec_reader* r);

/* ---- chunked wire messages (loggingModule.c:447-500, 299-354) ----------- */

/* Message sink: called once per message with the full message (header +
 * payload); return 0 to continue, non-zero to abort. */
typedef int (*youth_msg_sink)(void* user, const void* msg, size_t len);

/* Emit one frame as the logger's playback does (loggingModule.c:589-596):
 * a METADATA message, then the depth plane and the colour plane, each in
 * ceil(bytes / YOUTH_MSG_PAYLOAD) chunk messages.  color may be NULL (no
 * colour messages).  Returns the number of messages, or -1 if the sink aborted. */
int youth_wire_send_frame(youth_msg_sink sink, void* user, uint32_t frame_id,
                          uint32_t timestamp_ms, int width, int height, const int16_t* depth,
                          const uint8_t* color);

/* Frame reassembly from wire messages, following the logger's receive loop
 * (loggingModule.c:299-354): METADATA (re)sizes the planes; DEPTH/COLOR
 * chunks are copied at chunkIndex * YOUTH_MSG_PAYLOAD when they fit; a plane
 * is complete at its last chunk. */
typedef struct youth_frame_asm youth_frame_asm;
/* need_color = 1: a frame is complete when depth AND colour are (the
 * logger's rule); 0: when depth is (ICP needs no colour). */
youth_frame_asm* youth_asm_create(int need_color);
void youth_asm_destroy(youth_frame_asm* a);
/* Feed one message.  Returns 1 when it completed a frame (each frame is
 * reported once; *h, *depth, *color point into assembler-owned planes,
 * valid until the next call; *color is NULL if no colour arrived), 0
 * otherwise, -1 on a malformed message (too short, bad size). */
int youth_asm_push(youth_frame_asm* a, const void* msg, size_t len, youth_frame_header* h,
                   const int16_t** depth, const uint8_t** color);

/* ---- AlgorithmModule frame loop (SURVEY §8b thread entry) ---------------- */

/* Message source: copy the next message into buf (cap bytes) and return its
 * length, 0 if none arrived within timeout_ms, < 0 to end the loop. */
typedef int (*youth_msg_source)(void* user, void* buf, size_t cap, int timeout_ms);

/* The frame loop over any transport: pull messages from `recv`, reassemble
 * frames, processSlamFrame() each one, and hand every new trajectory pose to
 * `publish` (NULL: none) as one YOUTH_MSG_TYPE_POSE message.  Runs until recv
 * returns < 0, *stop becomes non-zero or the SLAM module stops.  *stop is
 * read with an atomic acquire load: set it from another thread with an
 * atomic store (e.g. __atomic_store_n(stop, 1, __ATOMIC_RELEASE)).  Returns
 * the number of frames handed to processSlamFrame. */
int youth_algorithm_run(youth_msg_source recv, void* recv_user, youth_msg_sink publish,
                        void* publish_user, volatile int* stop);

/* The same loop over POSIX queues: receive wire messages from `frame_queue` (created if absent, with the
 * reference's attributes), reassemble frames, processSlamFrame() each one,
 * and publish every new trajectory pose on `pose_queue` (NULL: none) as a
 * YOUTH_MSG_TYPE_POSE message.  Runs until *stop becomes non-zero (polled
 * every 50 ms) or the SLAM module stops.  Returns the number of frames
 * handed to processSlamFrame, or -1 if a queue could not be opened. */
int youth_algorithm_loop(const char* frame_queue, const char* pose_queue,
                         volatile int* stop);

/* Producer / consumer helpers over POSIX queues (opened with the reference's
 * attributes, created if absent): send one frame as METADATA + chunk
 * messages (blocking sends; the logger-side hand-off), and receive one pose
 * message (timeout_ms < 0: wait).  send: messages sent or -1; recv: 1 with
 * *h / *pose filled, 0 on timeout, -1 on error. */
int youth_wire_mq_send_frame(const char* queue, uint32_t frame_id, uint32_t timestamp_ms,
                             int width, int height, const int16_t* depth, const uint8_t* color);
int youth_wire_mq_recv_pose(const char* queue, int timeout_ms, youth_msg_header* h,
                            youth_pose_msg* pose);

/* Replay a recording through processSlamFrame (the f2 playback path; at the
 * logger's 30 fps pacing when realtime != 0).  Returns frames replayed, or -1. */
int youth_rec_play(const char* path, int realtime);

#ifdef __cplusplus
}
#endif

#endif /* YOUTH_WIRE_H */
