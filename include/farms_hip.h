/*
 * farms_hip.h — C ABI of libfarms_hip.so, the MI355X (gfx950) drop-in for the
 * FARMS_Flow batch hot path.
 *
 * The reference has no plugin registry or FFI: its boundary for this path is the
 * C++ class vFlowManager (/root/reference/include/vFlow.h:22-117), whose batch
 * method runFileCopy (/root/reference/src/vFlow.cpp:111-460) parses a text file,
 * runs the per-event loop (vFlow.cpp:223-414) and writes the _FARMSOut_ file.
 * This ABI replaces exactly that per-event loop; parsing, t0 subtraction,
 * polarity clamping, timing and the text writer stay in the host C++ mirror of
 * vFlowManager (host/vFlow.cpp), see INTEGRATION.md.
 *
 * Plain pointers and sizes only.  One handle per host thread; a handle owns one
 * HIP stream and the persistent sensor surfaces, so a stream of events may be fed
 * through several farms_process calls with results identical to one call.
 */
#ifndef FARMS_HIP_H
#define FARMS_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes */
#define FARMS_OK 0
#define FARMS_EINVAL (-1)  /* bad parameter, or an event outside the W x H sensor */
#define FARMS_EHIP (-2)    /* a HIP runtime call failed (message in farms_last_error) */
#define FARMS_ENOMEM (-3)  /* device or host allocation failed */
#define FARMS_ENODEV (-4)  /* no usable gfx950 device */
#define FARMS_EINTERNAL (-5) /* an internal ordering invariant of the engine failed (a bug; message in farms_last_error) */

typedef struct farms_handle farms_handle;

/* Constructor arguments of vFlowManager::vFlowManager(height, width, filterSize,
 * minEvtsOnPlane, fileName) (vFlow.h:100, vFlow.cpp:22-108), plus the two
 * constants the reference hard-codes at vFlow.cpp:73-74 (windowJump = 5,
 * maxWindow = 50; exposed for BASELINE config 5's 3-scale run) and placement. */
typedef struct {
    int32_t width;        /* --width  (vFlow.cpp:28) */
    int32_t height;       /* --height (vFlow.cpp:27) */
    int32_t filter_size;  /* --filtersize, normalised as vFlow.cpp:32-36 */
    int32_t min_inliers;  /* --inlierCheck = minEvtsOnPlane (vFlow.cpp:38) */
    int32_t window_jump;  /* pooling scale step, reference 5 */
    int32_t max_window;   /* largest pooling radius, reference 50 */
    int32_t device;       /* HIP device ordinal */
    int32_t fit_chunk;    /* events per local-fit chunk, 0 = default (65536) */
    int32_t pool_chunk;   /* events per pooling chunk, 0 = default (4096 where the stored region is at least about half of
                             1280x720; scaled down from 8192 (16384 at filtersize 7) on smaller regions) */
    /* spatial strips (multi-GPU): the handle stores columns [region_x0,
     * region_x0 + region_width) of the width x height sensor and pools only the
     * events of columns [own_x0, own_x1); events of the other stored columns are
     * fitted (their flows feed the owned events' pooling) and their r_true /
     * theta_true / scale are left 0.  region_width = 0: the whole sensor;
     * own_x1 = 0: every column.  With region = owned columns widened by
     * max_window + 1 + 2 * (filter_size / 2) on each side (clipped to the
     * sensor), owned records are bitwise those of a whole-sensor run. */
    int32_t region_x0, region_width;
    int32_t own_x0, own_x1;
    int32_t pool_batch;   /* pooling chunks per pooling launch, 0 = default (64; 32 at filtersize 7 on scaled-down
                             regions; with the 4096-event default chunk: 192, 64 at filtersize 7) */
    /* 1: the per-event semantics of vFlowManager::run (vFlow.cpp:465-826, the
     * CLI's --SERIAL 1, its default): lastEventTime is written after pooling
     * (:790), so an event's own cell is pooled with the stamp of the previous
     * event at its pixel (or farms_serial_first's), and an event with no
     * contributor takes its own flow at scale 0 (:1085-1094).  0: runFileCopy. */
    int32_t serial;
    /* 1: fit only the owned columns [own_x0, own_x1); the local flows of the
     * other stored events (the halo) are supplied by their owners through
     * farms_import_flows between farms_fit_device and farms_pool_device
     * (x-strips with a flow-halo exchange).  The stored region
     * must then cover the owned columns widened by max_window on the left and
     * max_window + floor(min(height - 1 + max_window, width - 1) / height) on the
     * right (the pooling window with the W-1 clip of vFlow.cpp:1000/1113). */
    int32_t import_halo;
} farms_params;

/* One output record per input event, the 11 columns of vFlow.cpp:438 in SoA
 * form: x y t p RTrue ThetaTrue Vx Vy RLocal ThetaLocal scale.  For
 * farms_process these are host arrays of length n; for farms_process_device
 * they are device arrays (x, y, t, p may be NULL there: they equal the inputs). */
typedef struct {
    int32_t *x, *y, *t, *p;
    double *r_true, *theta_true;
    double *vx, *vy;
    double *r_local, *theta_local;
    int32_t *scale;
} farms_records;

/* Counters of every farms_process* / farms_fit_device / farms_pool_device call
 * since the last farms_reset (or farms_create): asynchronous and pipelined calls
 * included.  farms_get_stats waits for the profiled work it reports. */
typedef struct {
    int64_t n_events;
    int64_t n_valid;         /* events that passed the validity gate (vFlow.cpp:315) */
    double sae_cells;        /* sum over events of U_loc */
    double pool_cells;       /* sum over valid events of U_pool */
    int32_t fit_launches, pool_launches;
    /* kernel time, ms, from HIP events on the handle's stream; filled only when
     * profiling is enabled (farms_set_profiling) */
    double ms_prep, ms_fit, ms_pool, ms_total;  /* phases: prep / fit sweep / pool sweep */
    double ms_fit_kernel;   /* sum of k_fit launch durations */
    double ms_pool_kernel;  /* sum of k_pool launch durations */
    double pool_candidates;   /* sum over valid events of candidate cells scanned */
    double pool_contributors; /* sum over valid events of contributing cells (largest scale) */
    int64_t n_owned;          /* events in the owned columns (all of them unless own_x1 is set) */
    /* wall time during which at least one k_fit (k_pool) launch runs: the union
     * of the launch brackets on the device timeline.  Equal to ms_fit_kernel
     * when the launches never overlap; below it when two fit streams run
     * launches side by side (fs 7), where the sum counts the overlap twice. */
    double ms_fit_busy, ms_pool_busy;
    /* the tail of the candidates scanned per pooled event (counting on, as
     * pool_candidates): the largest, and the events scanning more than 1,024 */
    int64_t pool_scan_max, pool_scan_over_1k;
} farms_stats;

/* vFlowManager ctor defaults: 320 x 320, filter 3, 5 inliers (main.cpp:21-24),
 * windowJump 5, maxWindow 50 (vFlow.cpp:73-74), device 0. */
int farms_default_params(farms_params *out);

int farms_create(const farms_params *params, farms_handle **out);
int farms_destroy(farms_handle *h);

/* Forget every event seen so far (fresh surfaces, as a new vFlowManager). */
int farms_reset(farms_handle *h);

/* Run the per-event loop of runFileCopy (vFlow.cpp:223-414) over n events in
 * stream order.  t_rel is T - t0 as uint32 (vFlow.cpp:240-241); p is the
 * polarity already clamped to >= 0 (vFlow.cpp:245-247) and is only echoed.
 * Host pointers; arrays in pinned memory (farms_host_alloc) are DMAed directly,
 * others through the handle's pinned staging.  Synchronous.  A long call runs
 * as a pipeline of sub-batches (bitwise one call); an event outside the sensor
 * returns FARMS_EINVAL before its sub-batch runs, earlier sub-batches of the
 * call having been processed (farms_reset to start over). */
int farms_process(farms_handle *h, const int32_t *x, const int32_t *y, const uint32_t *t_rel,
                  const int32_t *p, int64_t n, farms_records *out);

/* Pinned (page-locked) host memory for farms_process's inputs and records:
 * the DMA engines read and write it in place (no staging copy).  Not in the
 * reference (its vectors are pageable, vFlow.h:111-114). */
int farms_host_alloc(int64_t bytes, void **out);
int farms_host_free(void *p);

/* Same with device-resident inputs and outputs (no PCIe traffic).  Synchronous
 * with respect to the handle's stream.  At most 2^29 - 1 events per device call
 * (FARMS_EINVAL beyond; feed longer streams in pieces: split calls are bitwise
 * one call); farms_process cuts longer host calls itself. */
int farms_process_device(farms_handle *h, const int32_t *d_x, const int32_t *d_y,
                         const uint32_t *d_t_rel, const int32_t *d_p, int64_t n,
                         farms_records *d_out);

/* The per-event loop split at its one exchange point (x-strips):
 * farms_fit_device enqueues prep and the local fits (of the owned columns when
 * import_halo is set) over n device events; farms_export_flows (synchronous)
 * / farms_import_flows move the flows {L, L cos theta, L sin theta} (3 doubles
 * per listed event, d_idx = indices into those n events) out of / into the
 * handle for its oldest fit not yet pooled; farms_pool_device runs the pooling sweep of
 * the oldest fit not yet pooled into its records.  A stream may be fed in
 * sub-batches, and the fit (and exchange) of sub-batch b+1 may be issued before
 * the pooling of b (at most two fits pending): that pooling then runs
 * asynchronously under them; a farms_pool_device with no later fit pending
 * waits for the device.  Equivalent to farms_process_device when nothing is
 * imported.  Records of non-owned events are left unspecified; a halo flow
 * never imported counts as invalid.  An index outside [0, n) is skipped (no
 * device write through it); farms_export_flows / farms_export_wait and
 * farms_import_flows then return FARMS_EINVAL (the asynchronous import does
 * not wait, so it cannot report). */
int farms_fit_device(farms_handle *h, const int32_t *d_x, const int32_t *d_y, const uint32_t *d_t_rel,
                     const int32_t *d_p, int64_t n, farms_records *d_out);
int farms_export_flows(farms_handle *h, const int32_t *d_idx, int64_t count, double *d_flows);
int farms_import_flows(farms_handle *h, const int32_t *d_idx, int64_t count, const double *d_flows);
int farms_pool_device(farms_handle *h);

/* The same exchange without host waits on the device's other work, so that the
 * fit of sub-batch b+2 can be issued before the exchange of b+1 completes (the
 * x-strip pipeline): farms_export_flows_async enqueues the gather
 * behind the fit's work and returns; farms_export_wait returns once d_flows
 * holds it (waiting for nothing issued after the gather); farms_import_flows_async
 * enqueues the scatter ahead of that fit's pooling and returns at once -- d_flows
 * must stay valid and unchanged until the farms_pool_device of that fit has
 * completed.  All exchange calls act on the oldest fit not yet pooled. */
int farms_export_flows_async(farms_handle *h, const int32_t *d_idx, int64_t count, double *d_flows);
int farms_export_wait(farms_handle *h);
int farms_import_flows_async(farms_handle *h, const int32_t *d_idx, int64_t count, const double *d_flows);

/* Profiling of the next calls: FARMS_PROF_TIMING records HIP events around the
 * phases and every k_fit / k_pool launch on the stream that runs it (times in
 * farms_stats, summed over the calls since the last reset; ~1,700 event records
 * per 50M events), FARMS_PROF_POOL only around the
 * phases and the k_pool launches (ms_fit_kernel stays 0), FARMS_PROF_COUNTERS
 * also counts U_loc / U_pool / candidates / contributors (an extra kernel
 * pass, ~2% of a call).  0 = off (default); any other value = timing and
 * counters. */
#define FARMS_PROF_TIMING 1
#define FARMS_PROF_COUNTERS 2
#define FARMS_PROF_POOL 3
int farms_set_profiling(farms_handle *h, int enable);
int farms_get_stats(const farms_handle *h, farms_stats *out);

/* Copy the lastEventTime surface (vFlow.h:73, x-major W x H doubles: the stamp
 * of the latest event at each pixel, 0 if none) into host memory; the
 * reference exposes it as returnFlowTime() (vFlow.h:107). */
int farms_get_last_event_time(const farms_handle *h, double *out);

/* Temporal segments (multi-GPU on a time-ordered stream).  A
 * segment of the stream can be processed on its own, with results bitwise
 * those of the whole run, from (a) the SAE as of its first event and (b) the
 * local flows of the events of the last 500 us before it (re-fitted as a
 * warm-up prefix of the segment).  Stamp surfaces are x-major W x H int64
 * device arrays, -1 = pixel never visited.  Not in the reference (single
 * process); they feed an RCCL all-gather in bench.py. */

/* Last stamp per pixel over device events [0, n_head) -> d_head (may be NULL
 * when n_head = 0) and over [0, n) -> d_full. */
int farms_last_stamps(farms_handle *h, const int32_t *d_x, const int32_t *d_y, const uint32_t *d_t_rel,
                      int64_t n, int64_t n_head, int64_t *d_head, int64_t *d_full);
/* d_out[q] = the value of the last of the count arrays d_in[i * W * H + q]
 * that visited q (i.e. the SAE after the segments in order). */
int farms_merge_stamps(farms_handle *h, const int64_t *d_in, int32_t count, int64_t *d_out);
/* Start the handle (fresh or reset) from the SAE d_stamp; flow state stays empty. */
int farms_seed_sae(farms_handle *h, const int64_t *d_stamp);

/* Serial mode: the file's first line (x, y, absolute stamp t_abs) is not an
 * event of the loop; it only sets lastEventTime[x][y] = t_abs (vFlow.cpp:531-556).
 * Call once on a fresh (or reset) serial handle before farms_process. */
int farms_serial_first(farms_handle *h, int32_t x, int32_t y, uint32_t t_abs);

/* Number of pooling scales, floor(max_window / window_jump) + 1. */
int farms_num_scales(const farms_handle *h);

/* The kernels the handle's next call runs (its filter and scales, and the
 * FARMS_FIT_* / FARMS_POOL_* tuning knobs as they are now), and the candidate
 * build of the last pooling call enqueued (the host decides it when it
 * enqueues the call, from the prep's kill-window reach; this function does not
 * synchronise), as a JSON object in buf (NUL-terminated, truncated to len):
 * {"fit": "k_fit_quad<2>", "fit_mode": 1, "pool": "k_pool<11>", "pool_cap": 7,
 * "cand_last": "k_cand"}.  Not in the reference (measurement aid for bench.py). */
int farms_kernel_info(const farms_handle *h, char *buf, int32_t len);

/* Thread-local message for the last non-OK status. */
const char *farms_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
