// farms_engine.hip — MI355X (gfx950) implementation of the FARMS_Flow batch hot
// path behind the C ABI of include/farms_hip.h.
//
// What the reference does (src/vFlow.cpp:223-414), one event at a time:
//   SAE write -> computeLocalFlow (9-window plane fit, :841-949, :1214-1381)
//   -> validity gate (:315) -> flow-surface write -> computeTrueFlow (multiscale
//   pooling, :952-1210) -> record.
// Every event reads the surfaces as left by all earlier events and itself.
//
// How it runs here:
//   prep    pixel id per event; stable radix sort of event ids by pixel
//           (hipCUB) -> per-pixel runs in index order; prev/next links; a
//           second sort gives the work order (pooling chunk, 8x8 tile).
//   sweep 1 (local fit, stream F)  events in chunks of C1.  The SAE "as of
//           event e" at pixel q = the last event at q with index <= e: a
//           snapshot of the SAE at chunk start with the pixel's first two
//           in-chunk events inline (k_fit_prep), a run scan beyond that.
//           k_fit_quad: four lanes per event, the union of the 9 windows in
//           an LDS tile, exact integer scores and sums combined over the quad.
//   sweep 2 (pooling, streams C and P)  chunks of C2 in super-chunks of B.
//           k_chain keeps every cell's flow state in registers across the B
//           chunks and writes, per chunk, the candidate list (bitmap + group-
//           local slots) of cells that can contribute to any of its events;
//           k_pool pools one valid event per wavefront from that list.
// Local flow depends only on the SAE, pooling only on local flows and times, so
// these two sweeps reproduce the sequential semantics exactly.
//
// Numerics: fp64 throughout, compiled with -ffp-contract=off (no FMA), with the
// reference's (and Eigen 3.4's) evaluation order for the fit, and correctly
// rounded atan2 / sin / cos (farms_libm.h); see DESIGN.md §3.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <hipcub/block/block_radix_sort.hpp>

#include <algorithm>
#include <numeric>
#include <atomic>
#include <climits>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/farms_hip.h"
#include "farms_libm.h"

// correctly rounded atan2 / sincos (farms_libm.h)
#define F_ATAN2 farms_libm::cr_atan2
#define F_SINCOS farms_libm::cr_sincos

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(expr)                                                                   \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess)                                                          \
            return fail(e_ == hipErrorOutOfMemory ? FARMS_ENOMEM : FARMS_EHIP,         \
                        std::string(#expr) + ": " + hipGetErrorString(e_));            \
    } while (0)

constexpr double kMaxStamp = 4294967296.0;  // vFlow.h:27
constexpr double kTsToSec = 1e-6;           // vFlow.h:28
constexpr double kKillUs = 500.0;           // vFlow.cpp:961
constexpr int kDefaultFitChunk = 1 << 16;
constexpr int kDefaultPoolChunk = 1 << 13;
constexpr int kDefaultPoolBatch = 64;  // pooling chunks per super-chunk (ring of 3B+1 candidate buffers)
constexpr int kMaxScales = 16;

// Local-flow state of one event, and the flow surface cell (x-major).  L = 0 for
// an invalid event (vFlow.cpp:398-402); Lc/Ls = L*cos(theta), L*sin(theta), the
// per-visit products of vFlow.cpp:1007-1008 evaluated once per event.
struct __attribute__((aligned(32))) FlowCell {
    double L, Lc, Ls;
    uint32_t t;
    uint32_t pad;
};

// SAE cell (x-major): snapshot of the SAE at chunk start plus the first two
// events of the current chunk at this pixel, inline, so "stamp as of e" is
// resolved without pointer chasing unless the pixel fired three or more times
// in the chunk (a bar's ON/OFF pair is the common case).  Two arrays: the
// 12-B head, read by every window scan (a column of 13 cells is 156 B, loaded
// as dwordx3), and the 16-B tail, read only when a pixel fired twice in the
// chunk.
// head: tsnap: the snapshot stamp; t1: the first in-chunk event's stamp; w:
//   kHeadTouched = the pixel fired in the current fit chunk (e1, t1, the tail
//   are current; the chunk's prep sets it and clears it again when it commits
//   the pixel's last event to the snapshot, so no chunk sequence number is
//   kept), kHeadMore = more than one in-chunk event, kHeadVisited = the
//   snapshot is valid, bits 0..28 = e1, the first in-chunk event's id.
// tail: e2m: second in-chunk event id, bit31 = more than two (then the pixel's
//   run [run_lo, run_hi] of positions in P, scanned in PT, resolves later
//   events); t2: its stamp.
struct SaeHead {
    uint32_t tsnap;
    uint32_t t1;
    uint32_t w;
};
constexpr uint32_t kHeadTouched = 0x80000000u, kHeadMore = 0x40000000u, kHeadVisited = 0x20000000u;
constexpr uint32_t kHeadE1Mask = 0x1FFFFFFFu;
// events of one device call (their ids fit the head's 29 bits); farms_process
// cuts longer host calls into sub-batches below it
constexpr int64_t kMaxCallEvents = (int64_t)kHeadE1Mask;
struct __attribute__((aligned(16))) SaeTail {
    uint32_t e2m;
    uint32_t t2;
    int32_t run_lo, run_hi;
};
// One SAE buffer: WH heads and WH tails.
struct SaeBuf {
    SaeHead *head;
    SaeTail *tail;
};

// Pooling candidate: one cell of the per-chunk bitmap, its flow state before
// the chunk (snap) and after its first in-chunk event (one).  Split into a
// 16-B header read by every scan and a 48-B payload read only for contributors.
constexpr uint32_t kCandMore = 0x80000000u;     // > 1 event at the cell in the chunk
constexpr uint32_t kCandSnapOk = 0x40000000u;   // L_snap > 0
constexpr uint32_t kCandOneOk = 0x20000000u;    // L1 > 0
constexpr uint32_t kCandMore2 = 0x10000000u;    // > 2 events at the cell in the chunk
constexpr uint32_t kCandLinMask = 0x0FFFFFFFu;  // x-major cell index (W*H < 2^28)
struct __attribute__((aligned(16))) CandHdr {
    uint32_t lin;  // cell index | flags above
    int32_t e1;    // first in-chunk event at the cell, INT_MAX if untouched
    uint32_t t_snap, t1;
};
// One 64-cell word of a chunk's candidate bitmap with the candidate index of
// its first candidate: one 16-B load per lookup (k_pool's row setup reads three
// per window row, scattered over the window's columns).
struct __attribute__((aligned(16))) BmWord {
    uint64_t bm;
    uint32_t wo;
    uint32_t pad;
};
struct CandVal {
    double L_snap, Lc_snap, Ls_snap;
    double L1, Lc1, Ls1;
    // kCandMore2: the cell's in-chunk run [run_lo, run_hi] in P (a run search
    // resolves the state as of an event); exactly two in-chunk events: the
    // second one inline, run_lo = its event id | (its L > 0) << 31, run_hi = its
    // stamp, so that one dependent load replaces the search's three
    int32_t run_lo, run_hi;
};

constexpr uint32_t kSeqMask = 0x7FFFFFFFu;
// LDS packing of k_pool's row segments (32 bits each):
//   row segment = row << 25 | (candidate index - flattened index + kRowBias)
// valid while candidate slots stay below 2^24 (W * H <= kMaxSlots)
constexpr int kRowBias = 1 << 14;  // flattened positions of a window < 128 x 128
constexpr int64_t kMaxSlots = (int64_t(1) << 24) - 256;
// candidates per lane per pooling step (2, halving the scan's dependent round
// trips, took 20 more VGPRs and one wave per SIMD: C3 550.9 against 573
// Mevents/s, round 3)
constexpr int kPoolHalves = 1;
// k_pool staging: {L, L cos, L sin, 1} and k0 of the 64 x kPoolHalves entries of a step, 8-B words
// plus 8 slots for the entries a step carries to the next (the fold takes whole groups of 8)
constexpr int kPoolSlots = 64 * kPoolHalves + 8;
constexpr int kPoolValWords = 4 * kPoolSlots + kPoolSlots / 8;
constexpr int kPoolMaxM = 63;  // largest maxWindow (2M+1 rows <= 2 x 64 lanes; a row spans <= 2 candidate groups)
// k_pool's fold lanes (round 5): lane 4 kk + g holds quantity g of scale kk, so
// the members of an entry (scales k0..K-1) are the lanes >= 4 k0 and its mask
// comes from the scalar unit (fold8_salu).  Needs 4K < 64: the padding entries'
// 4K then selects junk lanes only.  Above (K = 16) the v_cmp fold (lane g K + kk).
#ifndef FARMS_POOL_SALU
#define FARMS_POOL_SALU 1  // tuning builds: 0 = the round-4 v_cmp fold for every K
#endif
template <int K>
constexpr bool kSaluFold = FARMS_POOL_SALU && 4 * K < 64;

// Diagnostic builds (make variant NAME=stamps DEFS=-DFARMS_POOL_STAMPS): k_pool
// reads the shader clock at its phase boundaries and adds each valid event's
// cycles per phase into g_pool_stamps (farms_debug_pool_stamps reads and
// clears them): [0] prologue (descriptor), [1] row setup, [2] candidate pass
// (fold included), [3] fold, [4] finish, [5] valid events, [6] steps, [7] fold
// groups.  The clock reads wait on the LDS counter too: a few % slower.
#ifdef FARMS_POOL_STAMPS
// per-wave sums in registers (pool_st), added by lane 0 at the wave's end into
// one of 1,024 slot rows (block % 1024: no contention on one address)
constexpr int kStampRows = 1024;
__device__ unsigned long long g_pool_stamps[8 * kStampRows];
struct PoolSt { uint64_t v[8]; };
#define POOL_CLOCK(v) const uint64_t v = (uint64_t)clock64()
#define POOL_STAMP_ADD(i, x) (pool_st.v[i] += (uint64_t)(x))
#else
#define POOL_CLOCK(v)
#define POOL_STAMP_ADD(i, x)
#endif

struct Ctx {
    int W, H, n;
    int64_t WH;            // cells stored by this handle (region columns x H)
    int64_t WHs;           // cells of the whole sensor (W x H): the pooling window's end
    int X0, XR1;           // stored region: columns [X0, XR1); cell index = (x - X0) * H + y
    int own_lo, own_hi;    // pooled (owned) columns [own_lo, own_hi)
    int fit_lo, fit_hi;    // fitted columns: all stored ones, or (import_halo) the owned ones
    bool fit_all;          // fit_lo / fit_hi cover the stored region (no per-event test)
    int fr, min_inl, J, M;
    float invJ;            // 1/J: scale index of a cell = floor((d + J - 1 + 0.5) * invJ)
    uint32_t kmagic;       // ceil(2^32 / J) (J > 1): ceil(d / J) = umulhi(d + J - 1, kmagic)
    const int32_t *x, *y, *p;
    const uint32_t *t;
    const uint32_t *pix;   // x*H + y per event
    const uint32_t *skey;  // pixel ids, sorted
    const int32_t *P;      // event ids sorted by (pixel, id)
    const int32_t *Q;      // event ids ordered by (pooling chunk, 8x8 tile): work order
    int4 *qe;              // per work-order position: {event id or -1 if not pooled, x, y, t} (k_pool_desc)
    int4 *fdesc;           // per work-order position: {event id, x, y, t} (k_fit_desc)
    // per event, one 16-B record (k_link): {position in P, previous and next
    // event at the pixel (-1 / INT_MAX: none), tpv}; tpv = the stamp the
    // pixel's SAE holds just before the event (the previous event's, or, for
    // the pixel's first event of the call, the snapshot's in serial mode, 0 in
    // batch mode, where it is not read)
    const int4 *link;
    SaeBuf cells;          // SAE snapshot + in-chunk first events, per cell (the fit chunk's buffer)
    const int2 *PT;        // per position in P: {event id, t}
    FlowCell *fsnap;       // flow snapshot
    int64_t *ftime;        // fsnap.L > 0 ? fsnap.t : -1  (bitmap pre-filter)
    FlowCell *evf;         // per-event local flow
    double2 *plane;        // per event: the fitted plane's slopes (a, b), from the fit to k_flow
    uint8_t *valid;
    int32_t *pcur, *pend;  // pooling sweep, per cell: cursor into the cell's run of P, last run position (-1: none)
    // ring of NB per-chunk candidate buffers (chunk ch uses buffer ch % NB):
    BmWord *bw_ring;       // candidate bitmap words + first candidate index (nwords per buffer)
    int nblk;              // candidate groups (kGroupCells cells each)
    int64_t cstride;       // candidate slots per buffer: nblk * kGroupCells
    CandHdr *hdr_ring;     // candidates of group g at [g * kGroupCells, ...), ascending cell index
    CandVal *val_ring;
    int64_t nwords;
    int NB, C2;            // ring size, events per pooling chunk
    int ring0;             // ring buffer of the call's first pooling chunk (chunk numbers continue across calls)
    int pool_bw, pool_rs;  // k_pool LDS per wave, in 8-B words: bitmap words, row segments
    const uint32_t *ctmin, *ctmax;  // per pooling chunk
    // event-driven candidate build (k_cand): per pooling chunk the first chunk
    // whose events can still be snapshots inside its kill window (cbk), the
    // call-start snapshot list {cell, stamp, first event of the call at the
    // cell}, the call's plan (kCi* below) and the per-(chunk, slice) scratch of
    // candidate items
    const int32_t *cbk;
    const int4 *slist;
    int *cinfo;
    int32_t *cscr;         // k_cand scratch: per chunk of a launch, WH item slots (a band's at its first cell)
    const int32_t *bstart; // k_cand: per pooling chunk, the work-order start of each column band (nbands + 1)
    // k_cand's S2 sources (k_cand_export): per (pooling chunk, column band),
    // its events that are the last at their cell in the chunk with a valid
    // flow, {event, cell, stamp, next event at the cell}, compacted to the
    // front of the band's work-order range, and their number (s2b, at the
    // band's bstart index)
    int4 *s2x;
    int32_t *s2b;
    int nbands, bandc;     // column bands, columns per band (bandc * H: whole candidate groups; a power of two)
    int band_slots;        // the call's candidate buffers hold k_cand's band-contiguous slots (else k_chain's)
    int tilesH, tshift;    // work-order tiles per column, log2 of the tile edge
    // serial mode (vFlowManager::run, vFlow.cpp:465-826): an event is pooled
    // with its pixel's lastEventTime still holding link.w, the stamp before it
    // (written only after pooling, :790)
    bool serial;
    // outputs
    double *vx, *vy, *r_local, *th_local, *r_true, *th_true;
    int32_t *scale;
    int32_t *ox, *oy, *ot, *op;
    unsigned long long *counters;  // [0] n_valid [1] sae cells [2] pool cells [3] cand [4] contrib [5] owned
    int2 *dbg_tc;                  // profiling only: per event (candidates scanned, contributors)
};

// ---------------------------------------------------------------------------
// as-of lookups.  Stamp of the last event with id <= e at a pixel that fired
// 3+ times in the chunk, given its second in-chunk event (run position
// lo + 1, stamp t2) is <= e: a short scan of the run's {id, t} pairs.
__device__ __forceinline__ uint32_t run_asof(const Ctx &c, int lo, int hi, int e, uint32_t t2) {
    uint32_t t = t2;
    for (int j = lo + 2; j <= hi; ++j) {
        const int2 pt = c.PT[j];
        if (pt.x > e) break;
        t = (uint32_t)pt.y;
    }
    return t;
}

// SAE stamp of pixel q as of event e: -1 never visited, else t.  h is the
// cell's head {tsnap, t1, w}; the tail (second event, run bounds) is loaded
// only when it decides the answer.  (seq: unused, the head's kHeadTouched
// marks in-chunk state of the current chunk.)
__device__ __forceinline__ int64_t sae_resolve_h(const Ctx &c, uint3 h, uint32_t q, int e, uint32_t seq) {
    (void)seq;
    if (h.z & kHeadTouched) {
        const int e1 = (int)(h.z & kHeadE1Mask);
        if (e1 <= e) {
            if (!(h.z & kHeadMore)) return (int64_t)h.y;
            const uint4 g = reinterpret_cast<const uint4 *>(c.cells.tail)[q];  // e2m, t2, run_lo, run_hi
            if ((int)(g.x & kSeqMask) > e) return (int64_t)h.y;
            if (!(g.x >> 31)) return (int64_t)g.y;
            return (int64_t)run_asof(c, (int)g.z, (int)g.w, e, g.y);
        }
    }
    return (h.z & kHeadVisited) ? (int64_t)h.x : int64_t(-1);
}

// Head-only resolution for the deferred form (fit_event_quad_u): when the
// tail decides (the pixel fired more than once in the chunk, its first
// in-chunk event at or before e), *defer is set and the first in-chunk stamp
// t1 is returned as a provisional value, which sae_fix_tail corrects after the
// scan.  Resolving those cells in place put a dependent tail load under a
// branch in every cell step, and the branch end waited for every load in
// flight: one serialized round trip per cell step whenever any lane of the
// wave needed its tail (with 131,072-event fit chunks, 16% of the touched
// pixels fire twice).
__device__ __forceinline__ int64_t sae_resolve_head(uint3 h, int e, bool &defer) {
    defer = false;
    if (h.z & kHeadTouched) {
        const int e1 = (int)(h.z & kHeadE1Mask);
        if (e1 <= e) {
            defer = (h.z & kHeadMore) != 0;
            return (int64_t)h.y;
        }
    }
    return (h.z & kHeadVisited) ? (int64_t)h.x : int64_t(-1);
}
// The same resolution in 32 bits (fit_event_quad_u): the stamp (0 for a
// never-visited cell, the reference's Event(0,0,0,0)), whether the cell is
// visited, and whether its tail decides (then the stamp is the provisional t1).
__device__ __forceinline__ uint32_t sae_head_stamp(uint3 h, int e, bool &vis, bool &defer) {
    const bool now = (int)h.z < 0 && (int)(h.z & kHeadE1Mask) <= e;  // touched, first in-chunk event <= e
    defer = now && (h.z & kHeadMore) != 0;
    const bool snap = (h.z & kHeadVisited) != 0;
    vis = now || snap;
    return now ? h.y : (snap ? h.x : 0u);
}
// The stamp as of e of a deferred cell q (its head says: touched, first event
// at or before e, more than one in-chunk event; t1 its first stamp), from the
// tail already loaded into g.
__device__ __forceinline__ uint32_t sae_fix_tail(const Ctx &c, uint4 g, uint32_t t1, int e) {
    if ((int)(g.x & kSeqMask) > e) return t1;
    if (!(g.x >> 31)) return g.y;
    return run_asof(c, (int)g.z, (int)g.w, e, g.y);
}

__device__ __forceinline__ uint3 sae_head(const Ctx &c, uint32_t q) {
    const SaeHead hd = c.cells.head[q];  // one dwordx3 load
    return make_uint3(hd.tsnap, hd.t1, hd.w);
}

__device__ __forceinline__ int64_t sae_asof(const Ctx &c, uint32_t q, int e, uint32_t seq) {
    return sae_resolve_h(c, sae_head(c, q), q, e, seq);
}

// XCD-aware work order: consecutive blocks are dealt round-robin to the 8
// XCDs (each with its own L2).  Block b instead takes logical block
// xcd_block(b, G), so that each XCD works through one contiguous range of the
// (tile-ordered) work and neighbouring events share an L2.  Bijective on [0, G).
__device__ __forceinline__ int xcd_block(int b, int G) {
    const int q = G >> 3, r = G & 7, x = b & 7;
    return x * q + (x < r ? x : r) + (b >> 3);
}
// Grouped variant: runs of 8 consecutive logical blocks stay on one XCD and
// the runs go round-robin over the XCDs (locality without uneven shares).
// Bijective on [0, G) when G is a multiple of 64; other grids keep blockIdx.
// consecutive fit blocks per XCD run (round 3, C3: runs of 16, 32 and 128
// blocks all within 0.3 ms of 8 per step; the L2 sharing of neighbouring
// tiles does not pace the fit)
constexpr int kFitRun = 8;
__device__ __forceinline__ int xcd_block_grouped(int b, int G) {
    constexpr int R = kFitRun;
    if (G % (8 * R)) return b;
    const int x = b & 7, i = b >> 3;  // XCD label, index within the XCD
    return (i / R) * (8 * R) + x * R + (i % R);
}
__device__ __forceinline__ int work_block() { return xcd_block((int)blockIdx.x, (int)gridDim.x); }
// ---------------------------------------------------------------------------
// prep

// Validate, pixel id, and the work-order key: (pooling chunk, 8x8 tile) so
// that the threads of a wave and the waves of a CU work on neighbouring pixels.
__global__ void k_prep(Ctx c, uint32_t *pix, int32_t *iota, uint32_t *wkey, int *err, int pool_chunk,
                       int tile_bits, int tile_shift) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= c.n) return;
    const int x = c.x[e], y = c.y[e];
    uint32_t tile = 0;
    if (x < c.X0 || x >= c.XR1 || y < 0 || y >= c.H) {
        atomicOr(err, 1);
        pix[e] = 0;
    } else {
        pix[e] = (uint32_t)(x - c.X0) * (uint32_t)c.H + (uint32_t)y;
        const int ts = tile_shift, tm = (1 << ts) - 1;
        tile = (uint32_t)((x - c.X0) >> ts) * (uint32_t)((c.H + tm) >> ts) + (uint32_t)(y >> ts);
    }
    wkey[e] = ((uint32_t)(e / pool_chunk) << tile_bits) | tile;
    iota[e] = e;
}

// Range check of a call's events (device arrays), on the copy stream: the
// host waits for it there instead of behind stream F's queue (where the prep of
// a two-phase fit waits for the pooling that last used its workspace set).
__global__ void k_validate(const int32_t *x, const int32_t *y, int n, int x0, int x1, int H, int *err) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    const int ex = x[e], ey = y[e];
    if (ex < x0 || ex >= x1 || ey < 0 || ey >= H) atomicOr(err, 1);
}

// Several device fills in one launch (farms_reset: the SAE, flow snapshots,
// per-set cursors and counters were thirteen hipMemsetAsync launches, about
// 0.1 ms of a 3.3-ms C2 step): segment i is words[i] 32-bit words of pattern
// pat[i] from p[i] (16-B aligned, as hipMalloc returns), stored 16 B at a time.
constexpr int kFillSegs = 16;
struct FillTable {
    void *p[kFillSegs];
    int64_t words[kFillSegs];
    uint32_t pat[kFillSegs];
    int n;
};
__global__ void k_fill(FillTable t) {
    const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, st = (int64_t)gridDim.x * blockDim.x;
    for (int k = 0; k < t.n; ++k) {
        const uint32_t v = t.pat[k];
        uint4 *q = static_cast<uint4 *>(t.p[k]);
        const int64_t nq = t.words[k] >> 2;
        for (int64_t i = i0; i < nq; i += st) q[i] = make_uint4(v, v, v, v);
        uint32_t *w = static_cast<uint32_t *>(t.p[k]);
        for (int64_t i = 4 * nq + i0; i < t.words[k]; i += st) w[i] = v;
    }
}

// Per position k of P (events sorted by pixel, then index): PT[k] = {event,
// stamp}, and the event's link record, one 16-B scatter per event.  The stamp
// of the previous position comes from the neighbouring lane.
__global__ void k_link(Ctx c, int4 *link, int2 *PT, bool serial) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const bool in = k < c.n;
    const int e = in ? c.P[k] : 0;
    const uint32_t te = in ? c.t[e] : 0u;
    uint32_t tp = (uint32_t)__shfl_up((int)te, 1, 64);
    if ((threadIdx.x & 63) == 0 && in && k > 0) tp = c.t[c.P[k - 1]];
    if (!in) return;
    const uint32_t q = c.skey[k];
    PT[k] = make_int2(e, (int)te);
    const bool first = !(k > 0 && c.skey[k - 1] == q), last = !(k + 1 < c.n && c.skey[k + 1] == q);
    // serial mode: lastEventTime[x][y] while e is pooled.  Before the call it
    // is the flow snapshot's stamp (the last event at q, 0 if none, or the
    // first line's stamp set by farms_serial_first); the pooling chain only
    // advances fsnap after prep.
    const uint32_t tpv = first ? (serial ? c.fsnap[q].t : 0u) : tp;
    link[e] = make_int4(k, first ? -1 : c.P[k - 1], last ? INT_MAX : c.P[k + 1], (int)tpv);
    if (first) c.pcur[q] = k;  // the pooling chain's run bounds of the cell
    if (last) c.pend[q] = k;
}

// per pooling chunk: min / max of t (general streams need not be time-sorted)
__global__ void k_chunk_minmax(const uint32_t *t, int n, int chunk, uint32_t *tmin, uint32_t *tmax) {
    const int ch = blockIdx.x;
    const int64_t b = (int64_t)ch * chunk;
    const int64_t e1 = b + chunk < n ? b + chunk : n;
    uint32_t lo = 0xFFFFFFFFu, hi = 0;
    for (int64_t e = b + threadIdx.x; e < e1; e += blockDim.x) {
        const uint32_t v = t[e];
        lo = v < lo ? v : lo;
        hi = v > hi ? v : hi;
    }
    __shared__ uint32_t slo[256], shi[256];
    slo[threadIdx.x] = lo;
    shi[threadIdx.x] = hi;
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
            slo[threadIdx.x] = min(slo[threadIdx.x], slo[threadIdx.x + s]);
            shi[threadIdx.x] = max(shi[threadIdx.x], shi[threadIdx.x + s]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        tmin[ch] = slo[0];
        tmax[ch] = shi[0];
    }
}

// Fit sweep, before chunk f (double-buffered SAE: chunk f reads buffer f % 2):
// for chunk f = [c0, c1), record at
// every touched pixel its first two in-chunk events inline and the bounds of
// its in-chunk run in P, and set the SAE snapshot to the pixel's last event
// before the chunk (prev of its first event); for the events [p0, c0) before
// it (chunks f-2 and f-1: the buffer last served chunk f-2), set the snapshot
// of the pixels they touched that chunk f does not touch to their last event.
// The two parts write disjoint cells.
__device__ __forceinline__ void fit_prep_thread(const Ctx &c, SaeBuf cells, int p0, int c0, int c1, uint32_t seq,
                                                int i) {
    const int ep = p0 + i;
    if (ep < c0) {
        const int nx = c.link[ep].z;
        if (nx >= c0 && nx >= c1) {  // last event of chunk f-1 at a pixel chunk f does not touch
            SaeHead *hd = &cells.head[c.pix[ep]];
            hd->w = kHeadVisited;  // committed: no longer touched (stale state of chunk f-2 cleared)
            hd->tsnap = c.t[ep];
        }
    }
    const int e = c0 + i;
    if (e >= c1) return;
    const uint32_t q = c.pix[e];
    const int4 lk = c.link[e];  // {pos, prev, next, stamp before}
    const int nx = lk.z;
    if (lk.y < c0) {  // first event of the pixel in the chunk
        SaeHead *hd = &cells.head[q];
        SaeTail *tl = &cells.tail[q];
        uint32_t vis = kHeadVisited;
        if (lk.y >= 0) hd->tsnap = (uint32_t)lk.w;
        else vis = hd->w & kHeadVisited;  // no earlier event in this call: keep the snapshot of earlier calls
        hd->w = vis | kHeadTouched | (nx < c1 ? kHeadMore : 0u) | (uint32_t)e;
        hd->t1 = c.t[e];
        // the tail is read only for a pixel that fires more than once in the
        // chunk (kHeadMore), and its run bounds only past a second event: a
        // pixel that fires once (84 % of them in fs 7's 65,536-event chunks)
        // leaves its tail's line untouched (scattered partial-line writes were
        // most of the prep's HBM traffic, 7.2 of 9.9 MB per C4 launch)
        if (nx < c1) {  // and the second one
            const int nn = c.link[nx].z;
            tl->e2m = (uint32_t)nx | (nn < c1 ? 0x80000000u : 0u);
            tl->t2 = c.t[nx];
            tl->run_lo = lk.x;
        }
    }
    if (nx >= c1 && lk.y >= c0) cells.tail[q].run_hi = lk.x;  // the last of two or more
}

// Pooling descriptors of work-order positions [p0, p1): {event, x, y, t}, the
// event -1 when it is not pooled here (invalid flow, or a halo event its owner
// pools), so that a pooling wave needs one load where it needed two dependent
// round trips (Q, then the event's fields).  Runs after the fits of the
// positions' chunks.
__global__ void k_pool_desc(Ctx c, int p0, int p1) {
    const int w = p0 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (w >= p1) return;
    const int4 fd = c.fdesc[w];
    const bool ok = c.valid[fd.x] && fd.y >= c.own_lo && fd.y < c.own_hi;
    c.qe[w] = make_int4(ok ? fd.x : -1, fd.y, fd.z, fd.w);
}

// Fit descriptor per work-order position: {event, x, y, t}, so that a fit
// wave opens with one 16-B load where it needed two dependent round trips (Q,
// then the event's fields).  After the work-order sort, in prep.
__global__ void k_fit_desc(Ctx c) {
    // XCD-contiguous blocks: a pooling chunk's gathers of x, y, t (its events
    // are a 8,192-event window) stay in one L2 instead of being fetched by all
    // eight (2.4 GB of fetches for 50M events with round-robin blocks, PMC)
    const int w = (int)(work_block() * blockDim.x + threadIdx.x);
    if (w >= c.n) return;
    const int e = c.Q[w];
    c.fdesc[w] = make_int4(e, c.x[e], c.y[e], (int)c.t[e]);
}

// The prep of one fit chunk as its own launch (the first chunk of a call, the
// final commits, the fit paths without a merged prep).
__global__ void k_fit_prep(Ctx c, SaeBuf cells, int p0, int c0, int c1, uint32_t seq) {
    fit_prep_thread(c, cells, p0, c0, c1, seq, (int)(blockIdx.x * blockDim.x + threadIdx.x));
}

// The prep of fit chunk f+1 riding on the launch of fit chunk f (blocks past
// the fit's grid; in the first blocks it measured slower, the fit sweep
// stretching 79 -> 83 ms at C3): it writes the other SAE buffer, which the fit
// of chunk f does not read, and the fit of chunk f-1 (the buffer's last reader)
// finished with the previous launch.
struct FitPrep {
    SaeBuf cells;
    int p0, c0, c1;
    uint32_t seq;
    int blocks;  // prep blocks after the fit's
};

// ---------------------------------------------------------------------------
// Eigen 3.4 PartialPivLU<MatrixXd>::determinant() of the 3x3 normal matrix
// (vFlow.cpp:1316); a is column-major (AtA.data()).  See oracle for the rules.
__device__ __forceinline__ double det3_partialpivlu(const double a[9]) {
    double m00 = a[0], m01 = a[3], m02 = a[6];
    double m10 = a[1], m11 = a[4], m12 = a[7];
    double m20 = a[2], m21 = a[5], m22 = a[8];
    int tr = 0;
    // k = 0
    {
        int piv = 0;
        double big = fabs(m00);
        if (fabs(m10) > big) { big = fabs(m10); piv = 1; }
        if (fabs(m20) > big) { big = fabs(m20); piv = 2; }
        if (big != 0.0) {
            if (piv == 1) { double t0 = m00, t1 = m01, t2 = m02; m00 = m10; m01 = m11; m02 = m12; m10 = t0; m11 = t1; m12 = t2; ++tr; }
            else if (piv == 2) { double t0 = m00, t1 = m01, t2 = m02; m00 = m20; m01 = m21; m02 = m22; m20 = t0; m21 = t1; m22 = t2; ++tr; }
            m10 = m10 / m00;
            m20 = m20 / m00;
        }
        m11 = m11 - m10 * m01; m12 = m12 - m10 * m02;
        m21 = m21 - m20 * m01; m22 = m22 - m20 * m02;
    }
    // k = 1
    {
        double big = fabs(m11);
        int piv = 1;
        if (fabs(m21) > big) { big = fabs(m21); piv = 2; }
        if (big != 0.0) {
            if (piv == 2) { double t0 = m10, t1 = m11, t2 = m12; m10 = m20; m11 = m21; m12 = m22; m20 = t0; m21 = t1; m22 = t2; ++tr; }
            m21 = m21 / m11;
        }
        m22 = m22 - m21 * m12;
    }
    const double prod = (m00 * m11) * m22;
    return (tr & 1) ? -prod : prod;
}

// ---------------------------------------------------------------------------
// Local plane fit of one event (computeLocalFlow + computeGrads, vFlow.cpp:
// 863-942, 1290-1380) for any fRad, every lookup complete, one thread.  Used
// for very large filters only (k_fit_wave stages smaller ones in LDS).
__device__ void fit_event_generic(const Ctx &c, int e, uint32_t seq, double &vx_out, double &vy_out, bool &acc_out) {
    const int fr = c.fr;
    const int side = 2 * fr + 1;
    const int np = side * side;
    const int W = c.W, H = c.H;
    const int ex = c.x[e], ey = c.y[e];
    const uint32_t te = c.t[e];
    vx_out = 0.0;
    vy_out = 0.0;
    acc_out = false;
    // ---- window scores (vFlow.cpp:870-912): sum over the window of
    // (t_e - t_k) + 2^32 [t_k > t_e], exact as int64; ties: first strict min.
    bool wok[9];
    int64_t score[9];
    bool any = false;
    for (int w = 0; w < 9; ++w) {
        const int ci = ex + (w / 3 - 1) * fr, cj = ey + (w % 3 - 1) * fr;
        wok[w] = ci - fr >= 0 && ci + fr <= W - 1 && cj - fr >= 0 && cj + fr <= H - 1;
        score[w] = 0;
        any |= wok[w];
    }
    if (!any) return;
    auto stamp = [&](int u, int v) -> int64_t {
        return (u >= c.X0 && u < c.XR1) ? sae_asof(c, (uint32_t)((u - c.X0) * H + v), e, seq) : int64_t(-1);
    };
    for (int du = -2 * fr; du <= 2 * fr; ++du) {
        const int u = ex + du;
        if (u < 0 || u >= W) continue;
        for (int dv = -2 * fr; dv <= 2 * fr; ++dv) {
            const int v = ey + dv;
            if (v < 0 || v >= H) continue;
            int mask = 0;
            for (int w = 0; w < 9; ++w) {
                const int ou = (w / 3 - 1) * fr, ov = (w % 3 - 1) * fr;
                if (du - ou <= fr && ou - du <= fr && dv - ov <= fr && ov - dv <= fr && wok[w]) mask |= 1 << w;
            }
            if (!mask) continue;
            const int64_t st = stamp(u, v);
            const uint32_t tk = st < 0 ? 0u : (uint32_t)st;
            const int64_t d = (int64_t)te - (int64_t)tk + (tk > te ? (int64_t(1) << 32) : 0);
            for (int w = 0; w < 9; ++w)
                if (mask & (1 << w)) score[w] += d;
        }
    }
    const int64_t nn = np;
    int64_t best = nn * ((int64_t(1) << 32) + 1);  // MAXSTAMP + 1 per cell
    int bw = -1;
    for (int w = 0; w < 9; ++w)
        if (wok[w] && score[w] < best) { best = score[w]; bw = w; }
    if (bw < 0 || best > nn * (int64_t(1) << 32)) return;
    // ---- the winning window, cx-major (vFlow.cpp:923-930)
    const int bi = ex + (bw / 3 - 1) * fr, bj = ey + (bw % 3 - 1) * fr;
    auto cell = [&](int k, int64_t &X, int64_t &Y, uint32_t &T) {
        const int cx = bi + k / side - fr, cy = bj + k % side - fr;
        const int64_t st = stamp(cx, cy);
        X = st >= 0 ? cx : 0; Y = st >= 0 ? cy : 0; T = st >= 0 ? (uint32_t)st : 0u;
    };
    int64_t sxx = 0, sxy = 0, sx = 0, syy = 0, sy = 0;
    for (int k = 0; k < np; ++k) {
        int64_t X, Y; uint32_t T;
        cell(k, X, Y, T);
        sxx += X * X; sxy += X * Y; sx += X; syy += Y * Y; sy += Y;
    }
    const double a[9] = {(double)sxx, (double)sxy, (double)sx, (double)sxy, (double)syy,
                         (double)sy,  (double)sx,  (double)sy, (double)np};  // AtA column-major (vFlow.cpp:1311)
    double DET = det3_partialpivlu(a);
    if (DET < 1) return;
    DET = 1.0 / DET;  // vFlow.cpp:1327-1336, A2 column-major
    const double d0 = DET * (a[8] * a[4] - a[7] * a[5]);
    const double d1 = DET * (a[7] * a[2] - a[8] * a[1]);
    const double d2 = DET * (a[5] * a[1] - a[4] * a[2]);
    const double d3 = DET * (a[6] * a[5] - a[8] * a[3]);
    const double d4 = DET * (a[8] * a[0] - a[6] * a[2]);
    const double d5 = DET * (a[3] * a[2] - a[5] * a[0]);
    const double d6 = DET * (a[7] * a[3] - a[6] * a[4]);
    const double d7 = DET * (a[6] * a[1] - a[7] * a[0]);
    const double d8 = DET * (a[4] * a[0] - a[3] * a[1]);
    // temp = (A2*At)*Y in Eigen's order
    const bool gemm = (3 + 3 + np) >= 20, gemv = (np + 3 + 1) >= 20;
    const double cz = (double)te * kTsToSec;
    double r0 = 0.0, r1 = 0.0, r2 = 0.0;
    for (int k = 0; k < np; ++k) {
        int64_t Xi, Yi; uint32_t T;
        cell(k, Xi, Yi, T);
        const double X = (double)Xi, Y = (double)Yi, Tk = (double)T;
        const double yt = T > te ? (Tk - kMaxStamp) * kTsToSec : Tk * kTsToSec;
        double m0, m1, m2;
        if (gemm) {
            m0 = (((0.0 + d0 * X) + d3 * Y) + d6 * 1.0) + 0.0;
            m1 = (((0.0 + d1 * X) + d4 * Y) + d7 * 1.0) + 0.0;
            m2 = (((0.0 + d2 * X) + d5 * Y) + d8 * 1.0) + 0.0;
        } else {
            m0 = (d0 * X + d3 * Y) + d6 * 1.0;
            m1 = (d1 * X + d4 * Y) + d7 * 1.0;
            m2 = (d2 * X + d5 * Y) + d8 * 1.0;
        }
        if (!gemv && k == 0) { r0 = m0 * yt; r1 = m1 * yt; r2 = m2 * yt; }
        else { r0 = r0 + m0 * yt; r1 = r1 + m1 * yt; r2 = r2 + m2 * yt; }
    }
    if (gemv) { r0 = r0 + 0.0; r1 = r1 + 0.0; r2 = r2 + 0.0; }
    (void)r2;
    const double dtdp = sqrt(r0 * r0 + r1 * r1);  // vFlow.cpp:1349-1377 (pow(v,2.0) as v*v)
    const double ccx = (double)ex, ccy = (double)ey;
    int inliers = 0;
    for (int k = 0; k < np; ++k) {
        int64_t Xi, Yi; uint32_t T;
        cell(k, Xi, Yi, T);
        const double Tk = (double)T;
        const double yt = T > te ? (Tk - kMaxStamp) * kTsToSec : Tk * kTsToSec;
        const double planedt = (r0 * ((double)Xi - ccx) + r1 * ((double)Yi - ccy));
        const double actualdt = yt - cz;
        if (fabs(planedt - actualdt) < dtdp / 2 && yt > 0) ++inliers;
    }
    if (inliers < c.min_inl) return;  // vFlow.cpp:934-942
    (void)dtdp;
    vx_out = r0;  // the plane's slopes: k_flow turns them into (Vx, Vy) (vFlow.cpp:1373-1377)
    vy_out = r1;
    acc_out = true;
}

// Local plane fit of one event with fRad known at compile time (the common
// filters 3, 5, 7): the union of the 9 candidate windows is loaded a column
// at a time and resolved from the inline in-chunk events; cells whose pixel
// fired 3+ times in the chunk (state past its second in-chunk event) are
// marked and resolved afterwards by a run search in a rolled loop, so the
// unrolled body stays small and no event leaves the kernel.  The winning
// window's stamps go to LDS (`lt`: this thread's column, stride 256) for the
// three passes over it.  Arithmetic is that of fit_event_generic.
template <int FR>
__device__ __forceinline__ void fit_event_fast(const Ctx &c, int4 fd, uint32_t seq, uint32_t *lt, double &vx_out,
                                               double &vy_out, bool &acc_out) {
    constexpr int side = 2 * FR + 1, np = side * side, US = 4 * FR + 1;
    const int W = c.W, H = c.H;
    const int e = fd.x, ex = fd.y, ey = fd.z;  // the fit descriptor (k_fit_desc)
    const uint32_t te = (uint32_t)fd.w;
    vx_out = 0.0;
    vy_out = 0.0;
    acc_out = false;
    bool wok[9];
    int64_t score[9];
    bool any = false;
#pragma unroll
    for (int w = 0; w < 9; ++w) {
        const int ci = ex + (w / 3 - 1) * FR, cj = ey + (w % 3 - 1) * FR;
        wok[w] = ci - FR >= 0 && ci + FR <= W - 1 && cj - FR >= 0 && cj + FR <= H - 1;
        score[w] = 0;
        any |= wok[w];
    }
    if (!any) return;
    // ---- window scores (vFlow.cpp:870-912), exact int64, first strict min.
    // The union window is walked a column at a time (two column buffers: the
    // next column's loads are in flight while this one is resolved); each
    // column's stamps give three vertical partial sums, which are added to the
    // windows whose column range contains it.  Every window's score is the
    // same integer sum in any order.
    auto load_col = [&](int u0, int v0, int len, uint3 *col) {
        const bool inr = u0 >= 0 && u0 < W && u0 >= c.X0 && u0 < c.XR1;  // outside the stored region: never visited
        const int cbase = (u0 - c.X0) * H + v0;
#pragma unroll
        for (int i = 0; i < len; ++i) {
            const int v = v0 + i;
            // unconditional load from a clamped index, then select: a load under a
            // branch is waited for at the branch's end, serializing the column
            const bool ok = inr && v >= 0 && v < H;
            const uint3 hd = sae_head(c, ok ? (uint32_t)(cbase + i) : 0u);
            col[i] = ok ? hd : make_uint3(0, 0, 0);
        }
    };
    auto score_col = [&](int du, const uint3 *col) {
        const int u = ex + du;
        if (u < 0 || u >= W) return;
        int64_t dd[US];
#pragma unroll
        for (int i = 0; i < US; ++i) {
            const int v = ey + i - 2 * FR;
            dd[i] = 0;
            if (v < 0 || v >= H) continue;
            const int64_t st = sae_resolve_h(c, col[i], (uint32_t)((u - c.X0) * H + v), e, seq);
            const uint32_t tk = st < 0 ? 0u : (uint32_t)st;
            dd[i] = (int64_t)te - (int64_t)tk + (tk > te ? (int64_t(1) << 32) : 0);
        }
#pragma unroll
        for (int ovi = 0; ovi < 3; ++ovi) {
            int64_t sv = 0;
#pragma unroll
            for (int i = ovi * FR; i <= ovi * FR + 2 * FR; ++i) sv += dd[i];
#pragma unroll
            for (int oui = 0; oui < 3; ++oui) {
                const int ou = (oui - 1) * FR;
                if (du - ou <= FR && ou - du <= FR) score[oui * 3 + ovi] += sv;
            }
        }
    };
#pragma unroll 1
    for (int du = -2 * FR; du <= 2 * FR; ++du) {
        uint3 ca[US];
        load_col(ex + du, ey - 2 * FR, US, ca);
        score_col(du, ca);
    }
    const int64_t nn = np;
    int64_t best = nn * ((int64_t(1) << 32) + 1);  // MAXSTAMP + 1 per cell
    int bw = -1;
#pragma unroll
    for (int w = 0; w < 9; ++w)
        if (wok[w] && score[w] < best) { best = score[w]; bw = w; }
    if (bw < 0 || best > nn * (int64_t(1) << 32)) return;

    // ---- gather the winning window, cx-major (vFlow.cpp:923-930), into LDS
    const int bi = ex + (bw / 3 - 1) * FR, bj = ey + (bw % 3 - 1) * FR;
    uint64_t vis = 0;
    auto gather_col = [&](int cxo, const uint3 *col) {
        const int u = bi + cxo - FR;
#pragma unroll
        for (int cyo = 0; cyo < side; ++cyo) {
            const int k = cxo * side + cyo;
            const int64_t st = sae_resolve_h(c, col[cyo], (uint32_t)((u - c.X0) * H + bj - FR + cyo), e, seq);
            vis |= st >= 0 ? 1ull << k : 0ull;
            lt[k * 256] = st < 0 ? 0u : (uint32_t)st;
        }
    };
#pragma unroll 1
    for (int cxo = 0; cxo < side; ++cxo) {
        uint3 ga[side];
        load_col(bi - FR + cxo, bj - FR, side, ga);
        gather_col(cxo, ga);
    }
    auto cell = [&](int k, int64_t &X, int64_t &Y, uint32_t &T) {
        const int cx = bi + k / side - FR, cy = bj + k % side - FR;
        const bool vk = (vis >> k) & 1;
        X = vk ? cx : 0; Y = vk ? cy : 0; T = lt[k * 256];
    };
    int64_t sxx = 0, sxy = 0, sx = 0, syy = 0, sy = 0;
#pragma unroll 1
    for (int k = 0; k < np; ++k) {
        int64_t X, Y; uint32_t T;
        cell(k, X, Y, T);
        sxx += X * X; sxy += X * Y; sx += X; syy += Y * Y; sy += Y;
    }
    const double a[9] = {(double)sxx, (double)sxy, (double)sx, (double)sxy, (double)syy,
                         (double)sy,  (double)sx,  (double)sy, (double)np};
    double DET = det3_partialpivlu(a);
    if (DET < 1) return;  // 0 inliers
    DET = 1.0 / DET;  // vFlow.cpp:1327-1336, A2 column-major
    const double d0 = DET * (a[8] * a[4] - a[7] * a[5]);
    const double d1 = DET * (a[7] * a[2] - a[8] * a[1]);
    const double d2 = DET * (a[5] * a[1] - a[4] * a[2]);
    const double d3 = DET * (a[6] * a[5] - a[8] * a[3]);
    const double d4 = DET * (a[8] * a[0] - a[6] * a[2]);
    const double d5 = DET * (a[3] * a[2] - a[5] * a[0]);
    const double d6 = DET * (a[7] * a[3] - a[6] * a[4]);
    const double d7 = DET * (a[6] * a[1] - a[7] * a[0]);
    const double d8 = DET * (a[4] * a[0] - a[3] * a[1]);
    constexpr bool gemm = (3 + 3 + np) >= 20, gemv = (np + 3 + 1) >= 20;
    const double cz = (double)te * kTsToSec;
    double r0 = 0.0, r1 = 0.0, r2 = 0.0;
#pragma unroll 1
    for (int k = 0; k < np; ++k) {
        int64_t Xi, Yi; uint32_t T;
        cell(k, Xi, Yi, T);
        const double X = (double)Xi, Y = (double)Yi, Tk = (double)T;
        const double yt = T > te ? (Tk - kMaxStamp) * kTsToSec : Tk * kTsToSec;
        double m0, m1, m2;
        if (gemm) {
            m0 = (((0.0 + d0 * X) + d3 * Y) + d6 * 1.0) + 0.0;
            m1 = (((0.0 + d1 * X) + d4 * Y) + d7 * 1.0) + 0.0;
            m2 = (((0.0 + d2 * X) + d5 * Y) + d8 * 1.0) + 0.0;
        } else {
            m0 = (d0 * X + d3 * Y) + d6 * 1.0;
            m1 = (d1 * X + d4 * Y) + d7 * 1.0;
            m2 = (d2 * X + d5 * Y) + d8 * 1.0;
        }
        if (!gemv && k == 0) { r0 = m0 * yt; r1 = m1 * yt; r2 = m2 * yt; }
        else { r0 = r0 + m0 * yt; r1 = r1 + m1 * yt; r2 = r2 + m2 * yt; }
    }
    if (gemv) { r0 = r0 + 0.0; r1 = r1 + 0.0; r2 = r2 + 0.0; }
    (void)r2;
    const double dtdp = sqrt(r0 * r0 + r1 * r1);  // vFlow.cpp:1349-1377 (pow(v,2.0) as v*v)
    const double ccx = (double)ex, ccy = (double)ey;
    int inliers = 0;
#pragma unroll 1
    for (int k = 0; k < np; ++k) {
        int64_t Xi, Yi; uint32_t T;
        cell(k, Xi, Yi, T);
        const double Tk = (double)T;
        const double yt = T > te ? (Tk - kMaxStamp) * kTsToSec : Tk * kTsToSec;
        const double planedt = (r0 * ((double)Xi - ccx) + r1 * ((double)Yi - ccy));
        const double actualdt = yt - cz;
        if (fabs(planedt - actualdt) < dtdp / 2 && yt > 0) ++inliers;
    }
    if (inliers < c.min_inl) return;  // vFlow.cpp:934-942
    (void)dtdp;
    vx_out = r0;  // the plane's slopes: k_flow turns them into (Vx, Vy) (vFlow.cpp:1373-1377)
    vy_out = r1;
    acc_out = true;
}

// Validity gate, flow-surface value and record of one fitted event.
__device__ __forceinline__ void fit_store(const Ctx &c, int e, double vx, double vy) {
    const uint32_t te = c.t[e];
    const int ex = c.x[e], ey = c.y[e];
    // ---- validity gate and flow-surface value (vFlow.cpp:315-357, 384-403)
    const bool ok = !isnan(fabs(vx)) && !isnan(fabs(vy)) && vx != 0 && vy != 0;
    FlowCell f;
    f.t = te;
    f.pad = 0;
    double L = 0.0, th = 0.0;
    if (ok) {
        L = sqrt(vx * vx + vy * vy);
        th = F_ATAN2(vy, vx);
        f.L = L;
        double sn_, cs_;
        F_SINCOS(th, &sn_, &cs_);
        f.Lc = L * cs_;
        f.Ls = L * sn_;
    } else {
        f.L = 0.0; f.Lc = 0.0; f.Ls = 0.0;
    }
    c.evf[e] = f;
    c.valid[e] = ok ? 1 : 0;
    c.vx[e] = vx;
    c.vy[e] = vy;
    c.r_local[e] = L;
    c.th_local[e] = th;
    if (!ok) { c.r_true[e] = 0.0; c.th_true[e] = 0.0; c.scale[e] = 0; }
    if (c.ox) { c.ox[e] = ex; c.oy[e] = ey; c.ot[e] = (int32_t)te; c.op[e] = c.p[e]; }
}

// The fit kernels end at the plane: its slopes (a, b) and whether the window
// search, the determinant and the inlier count accepted it (in c.valid until
// k_flow writes the validity there).  The libm chain that turns them into the
// local flow runs in k_flow, one lane per event, instead of on a quad's four
// lanes (or one of them) inside the fit.
__device__ __forceinline__ void fit_plane(const Ctx &c, int e, double r0, double r1, bool acc) {
    c.plane[e] = make_double2(r0, r1);
    c.valid[e] = acc ? 1 : 0;
}

// Local flow of events [e0, e1) from their planes (vFlow.cpp:1349-1377, then
// the validity gate and flow-surface value, fit_store): speed = 1 / |(a, b)|,
// angle = atan2(a, b), (Vx, Vy) = speed (cos, sin)(angle); (0, 0) when the plane
// was rejected.  Halo events of an x-strip (not fitted here) are left to
// farms_import_flows.
__global__ void k_flow(Ctx c, int e0, int e1) {
    const int e = e0 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (e >= e1) return;
    if (!c.fit_all) {
        const int ex = c.x[e];
        if (ex < c.fit_lo || ex >= c.fit_hi) {
            // a halo event: invalid until farms_import_flows supplies its
            // owner's flow (a flow never imported is not pooled, never stale)
            FlowCell f;
            f.L = 0.0; f.Lc = 0.0; f.Ls = 0.0; f.t = c.t[e]; f.pad = 0;
            c.evf[e] = f;
            c.valid[e] = 0;
            return;
        }
    }
    double vx = 0.0, vy = 0.0;
    if (c.valid[e]) {
        const double2 pl = c.plane[e];
        const double r0 = pl.x, r1 = pl.y;
        const double dtdp = sqrt(r0 * r0 + r1 * r1);  // pow(v, 2.0) as v*v
        const double speed = 1.0 / dtdp;
        const double angle = F_ATAN2(r0, r1);
        double sn_, cs_;
        F_SINCOS(angle, &sn_, &cs_);  // one range reduction for both
        vx = speed * cs_;
        vy = speed * sn_;
    }
    fit_store(c, e, vx, vy);
}

// One thread per event of chunk [c0, c1) in tile order.
template <int FR>
__global__ __launch_bounds__(256) void k_fit(Ctx c, int c0, int c1, uint32_t seq) {
    constexpr int NPC = (2 * FR + 1) * (2 * FR + 1);
    __shared__ uint32_t s_tk[NPC * 256];
    const int w = c0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= c1) return;
    const int4 fd = c.fdesc[w];  // chunk [c0, c1) occupies positions [c0, c1) of Q
    if (!c.fit_all && (fd.y < c.fit_lo || fd.y >= c.fit_hi)) return;
    double vx, vy;
    bool acc;
    fit_event_fast<FR>(c, fd, seq, s_tk + threadIdx.x, vx, vy, acc);
    fit_plane(c, fd.x, vx, vy, acc);
}


// ---------------------------------------------------------------------------
// Cross-lane exchange with the partner lane l ^ (1 << S): DPP quad
// permutations for S = 0, 1, ds_swizzle (bitmask mode, 32-lane groups) for
// S = 2..4, ds_bpermute for S = 5.
template <int S>
__device__ __forceinline__ int xch32(int v) {
    if constexpr (S == 0) return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true);  // quad_perm [1,0,3,2]
    else if constexpr (S == 1) return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, true);  // quad_perm [2,3,0,1]
    else if constexpr (S == 2) return __builtin_amdgcn_ds_swizzle(v, 0x101F);
    else if constexpr (S == 3) return __builtin_amdgcn_ds_swizzle(v, 0x201F);
    else if constexpr (S == 4) return __builtin_amdgcn_ds_swizzle(v, 0x401F);
    else return __shfl_xor(v, 32, 64);
}
// lane U of the quad, to every lane of the quad (DPP quad_perm [U,U,U,U])
template <int U>
__device__ __forceinline__ double quad_bcast(double v) {
    constexpr int ctl = U | (U << 2) | (U << 4) | (U << 6);
    return __hiloint2double(__builtin_amdgcn_mov_dpp(__double2hiint(v), ctl, 0xF, 0xF, true),
                            __builtin_amdgcn_mov_dpp(__double2loint(v), ctl, 0xF, 0xF, true));
}
template <int S>
__device__ __forceinline__ double xch(double v) {
    return __hiloint2double(xch32<S>(__double2hiint(v)), xch32<S>(__double2loint(v)));
}

// ---------------------------------------------------------------------------
// Quad-cooperative fit (fRad known at compile time): four lanes per event, so
// a 64k-event fit chunk is 4096 wavefronts and each lane issues a quarter of
// the dependent column loads.  Lane j of the quad scores union columns
// du = -2fRad + j, +4, ... and gathers window columns j, j + 4, ...; the
// integer window scores, the visited mask and the normal-matrix sums are
// combined with quad DPP exchanges (exact), the inlier count likewise.  The
// order-sensitive (A2*At)*Y accumulation runs in full on every lane of the
// quad from the window stamps in LDS, in the reference order, so all four
// lanes hold the bitwise result of the per-thread path.
__device__ __forceinline__ int64_t quad_sum_i64(int64_t v) {
    int hi = (int)(v >> 32), lo = (int)(uint32_t)v;
    int64_t o = ((int64_t)xch32<0>(hi) << 32) | (uint32_t)xch32<0>(lo);
    v += o;
    hi = (int)(v >> 32); lo = (int)(uint32_t)v;
    o = ((int64_t)xch32<1>(hi) << 32) | (uint32_t)xch32<1>(lo);
    return v + o;
}
__device__ __forceinline__ uint64_t quad_or_u64(uint64_t v) {
    int hi = (int)(v >> 32), lo = (int)(uint32_t)v;
    v |= ((uint64_t)(uint32_t)xch32<0>(hi) << 32) | (uint32_t)xch32<0>(lo);
    hi = (int)(v >> 32); lo = (int)(uint32_t)v;
    return v | ((uint64_t)(uint32_t)xch32<1>(hi) << 32) | (uint32_t)xch32<1>(lo);
}

// one-wave k_fit_quad workgroups (16 events each): a finished wave frees its
// slot at once (4-wave groups held it for their slowest event)
constexpr int kFitQS = 16;  // quads per fit workgroup: stride of the LDS stamp tiles

template <int FR>
__device__ __forceinline__ void fit_event_quad(const Ctx &c, int4 fd, uint32_t seq, int j, uint32_t *lt, double &vx_out,
                                               double &vy_out, bool &acc_out) {
    constexpr int side = 2 * FR + 1, np = side * side, US = 4 * FR + 1;
    const int W = c.W, H = c.H;
    const int e = fd.x, ex = fd.y, ey = fd.z;  // the fit descriptor (k_fit_desc)
    const uint32_t te = (uint32_t)fd.w;
    vx_out = 0.0;
    vy_out = 0.0;
    acc_out = false;
    bool wok[9];
    int64_t score[9];
    bool any = false;
#pragma unroll
    for (int w = 0; w < 9; ++w) {
        const int ci = ex + (w / 3 - 1) * FR, cj = ey + (w % 3 - 1) * FR;
        wok[w] = ci - FR >= 0 && ci + FR <= W - 1 && cj - FR >= 0 && cj + FR <= H - 1;
        score[w] = 0;
        any |= wok[w];
    }
    if (!any) return;  // uniform over the quad
    auto load_col = [&](int u0, int v0, int len, uint3 *col) {
        const bool inr = u0 >= 0 && u0 < W && u0 >= c.X0 && u0 < c.XR1;  // outside the stored region: never visited
        const int cbase = (u0 - c.X0) * H + v0;
#pragma unroll
        for (int i = 0; i < len; ++i) {
            const int v = v0 + i;
            // unconditional load from a clamped index, then select: a load under a
            // branch is waited for at the branch's end, serializing the column
            const bool ok = inr && v >= 0 && v < H;
            const uint3 hd = sae_head(c, ok ? (uint32_t)(cbase + i) : 0u);
            col[i] = ok ? hd : make_uint3(0, 0, 0);
        }
    };
    // ---- window scores (vFlow.cpp:870-912), exact int64: this lane's union
    // columns; cells whose tail decides take their first in-chunk stamp and
    // are corrected after the scan (sae_resolve_head)
    auto ddiff = [&](uint32_t tk) { return (int64_t)te - (int64_t)tk + (tk > te ? (int64_t(1) << 32) : 0); };
    uint64_t pend = 0;  // deferred cells: bit (column slot) * US + row
#pragma unroll 1
    for (int du = -2 * FR + j; du <= 2 * FR; du += 4) {
        uint3 col[US];
        load_col(ex + du, ey - 2 * FR, US, col);
        const int u = ex + du;
        if (u < 0 || u >= W) continue;
        const int sl = (du + 2 * FR) >> 2;
        int64_t dd[US];
#pragma unroll
        for (int i = 0; i < US; ++i) {
            const int v = ey + i - 2 * FR;
            dd[i] = 0;
            if (v < 0 || v >= H) continue;
            bool defer;
            const int64_t st = sae_resolve_head(col[i], e, defer);
            pend |= defer ? 1ull << (sl * US + i) : 0ull;
            const uint32_t tk = st < 0 ? 0u : (uint32_t)st;
            dd[i] = ddiff(tk);
        }
#pragma unroll
        for (int ovi = 0; ovi < 3; ++ovi) {
            int64_t sv = 0;
#pragma unroll
            for (int i = ovi * FR; i <= ovi * FR + 2 * FR; ++i) sv += dd[i];
#pragma unroll
            for (int oui = 0; oui < 3; ++oui) {
                const int ou = (oui - 1) * FR;
                if (du - ou <= FR && ou - du <= FR) score[oui * 3 + ovi] += sv;
            }
        }
    }
    // the deferred cells: head (its t1) and tail, four cells in flight at a time
#pragma unroll 1
    while (pend) {
        int bit[4];
        uint3 hh[4];
        uint4 g[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            bit[k] = pend ? (int)__builtin_ctzll(pend) : -1;
            pend &= pend ? pend - 1 : 0ull;
            const int b = bit[k] < 0 ? 0 : bit[k];
            const uint32_t q = bit[k] < 0 ? 0u : (uint32_t)((ex + j + 4 * (b / US) - 2 * FR - c.X0) * H + ey + b % US - 2 * FR);
            hh[k] = sae_head(c, q);
            g[k] = reinterpret_cast<const uint4 *>(c.cells.tail)[q];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (bit[k] < 0) continue;
            const uint32_t t1 = hh[k].y, tk = sae_fix_tail(c, g[k], t1, e);
            if (tk == t1) continue;
            const int64_t delta = ddiff(tk) - ddiff(t1);
            const int du = j + 4 * (bit[k] / US) - 2 * FR, i = bit[k] % US;
#pragma unroll
            for (int w = 0; w < 9; ++w) {
                const int ou = (w / 3 - 1) * FR, ovi = w % 3;
                if (du - ou <= FR && ou - du <= FR && i >= ovi * FR && i <= ovi * FR + 2 * FR) score[w] += delta;
            }
        }
    }
#pragma unroll
    for (int w = 0; w < 9; ++w) score[w] = quad_sum_i64(score[w]);
    const int64_t nn = np;
    int64_t best = nn * ((int64_t(1) << 32) + 1);  // MAXSTAMP + 1 per cell
    int bw = -1;
#pragma unroll
    for (int w = 0; w < 9; ++w)
        if (wok[w] && score[w] < best) { best = score[w]; bw = w; }
    if (bw < 0 || best > nn * (int64_t(1) << 32)) return;  // uniform over the quad

    // ---- gather the winning window, cx-major (vFlow.cpp:923-930): this lane's
    // columns into LDS (lt[k * kFitQS]), visited mask combined over the quad;
    // deferred cells again corrected after the pass
    const int bi = ex + (bw / 3 - 1) * FR, bj = ey + (bw % 3 - 1) * FR;
    uint64_t vis = 0, pend2 = 0;
#pragma unroll 1
    for (int cxo = j; cxo < side; cxo += 4) {
        uint3 col[side];
        load_col(bi - FR + cxo, bj - FR, side, col);
#pragma unroll
        for (int cyo = 0; cyo < side; ++cyo) {
            const int k = cxo * side + cyo;
            bool defer;
            const int64_t st = sae_resolve_head(col[cyo], e, defer);
            vis |= st >= 0 ? 1ull << k : 0ull;
            pend2 |= defer ? 1ull << k : 0ull;
            lt[k * kFitQS] = st < 0 ? 0u : (uint32_t)st;
        }
    }
#pragma unroll 1
    while (pend2) {
        int kk[4];
        uint4 g[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            kk[m] = pend2 ? (int)__builtin_ctzll(pend2) : -1;
            pend2 &= pend2 ? pend2 - 1 : 0ull;
            const int k = kk[m] < 0 ? 0 : kk[m];
            const uint32_t q = kk[m] < 0 ? 0u : (uint32_t)((bi + k / side - FR - c.X0) * H + bj + k % side - FR);
            g[m] = reinterpret_cast<const uint4 *>(c.cells.tail)[q];
        }
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            if (kk[m] < 0) continue;
            uint32_t *slot = &lt[kk[m] * kFitQS];
            *slot = sae_fix_tail(c, g[m], *slot, e);
        }
    }
    vis = quad_or_u64(vis);
    // the window's stamps were written by the other lanes of this wave's quad
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    auto cell = [&](int k, int64_t &X, int64_t &Y, uint32_t &T) {
        const int cx = bi + k / side - FR, cy = bj + k % side - FR;
        const bool vk = (vis >> k) & 1;
        X = vk ? cx : 0; Y = vk ? cy : 0; T = lt[k * kFitQS];
    };
    int64_t sxx = 0, sxy = 0, sx = 0, syy = 0, sy = 0;  // exact: any split and order
#pragma unroll 1
    for (int k = j; k < np; k += 4) {
        int64_t X, Y; uint32_t T;
        cell(k, X, Y, T);
        sxx += X * X; sxy += X * Y; sx += X; syy += Y * Y; sy += Y;
    }
    sxx = quad_sum_i64(sxx); sxy = quad_sum_i64(sxy); sx = quad_sum_i64(sx);
    syy = quad_sum_i64(syy); sy = quad_sum_i64(sy);
    const double a[9] = {(double)sxx, (double)sxy, (double)sx, (double)sxy, (double)syy,
                         (double)sy,  (double)sx,  (double)sy, (double)np};
    double DET = det3_partialpivlu(a);
    if (DET < 1) return;  // 0 inliers; uniform over the quad
    DET = 1.0 / DET;  // vFlow.cpp:1327-1336, A2 column-major
    const double d0 = DET * (a[8] * a[4] - a[7] * a[5]);
    const double d1 = DET * (a[7] * a[2] - a[8] * a[1]);
    const double d2 = DET * (a[5] * a[1] - a[4] * a[2]);
    const double d3 = DET * (a[6] * a[5] - a[8] * a[3]);
    const double d4 = DET * (a[8] * a[0] - a[6] * a[2]);
    const double d5 = DET * (a[3] * a[2] - a[5] * a[0]);
    const double d6 = DET * (a[7] * a[3] - a[6] * a[4]);
    const double d7 = DET * (a[6] * a[1] - a[7] * a[0]);
    const double d8 = DET * (a[4] * a[0] - a[3] * a[1]);
    constexpr bool gemm = (3 + 3 + np) >= 20, gemv = (np + 3 + 1) >= 20;
    const double cz = (double)te * kTsToSec;
    double r0 = 0.0, r1 = 0.0, r2 = 0.0;
#pragma unroll 1
    for (int k = 0; k < np; ++k) {  // every lane, reference order
        int64_t Xi, Yi; uint32_t T;
        cell(k, Xi, Yi, T);
        const double X = (double)Xi, Y = (double)Yi, Tk = (double)T;
        const double yt = T > te ? (Tk - kMaxStamp) * kTsToSec : Tk * kTsToSec;
        double m0, m1, m2;
        if (gemm) {
            m0 = (((0.0 + d0 * X) + d3 * Y) + d6 * 1.0) + 0.0;
            m1 = (((0.0 + d1 * X) + d4 * Y) + d7 * 1.0) + 0.0;
            m2 = (((0.0 + d2 * X) + d5 * Y) + d8 * 1.0) + 0.0;
        } else {
            m0 = (d0 * X + d3 * Y) + d6 * 1.0;
            m1 = (d1 * X + d4 * Y) + d7 * 1.0;
            m2 = (d2 * X + d5 * Y) + d8 * 1.0;
        }
        if (!gemv && k == 0) { r0 = m0 * yt; r1 = m1 * yt; r2 = m2 * yt; }
        else { r0 = r0 + m0 * yt; r1 = r1 + m1 * yt; r2 = r2 + m2 * yt; }
    }
    if (gemv) { r0 = r0 + 0.0; r1 = r1 + 0.0; r2 = r2 + 0.0; }
    (void)r2;
    const double dtdp = sqrt(r0 * r0 + r1 * r1);  // vFlow.cpp:1349-1377 (pow(v,2.0) as v*v)
    const double ccx = (double)ex, ccy = (double)ey;
    int inliers = 0;
#pragma unroll 1
    for (int k = j; k < np; k += 4) {
        int64_t Xi, Yi; uint32_t T;
        cell(k, Xi, Yi, T);
        const double Tk = (double)T;
        const double yt = T > te ? (Tk - kMaxStamp) * kTsToSec : Tk * kTsToSec;
        const double planedt = (r0 * ((double)Xi - ccx) + r1 * ((double)Yi - ccy));
        const double actualdt = yt - cz;
        if (fabs(planedt - actualdt) < dtdp / 2 && yt > 0) ++inliers;
    }
    inliers += xch32<0>(inliers);
    inliers += xch32<1>(inliers);
    if (inliers < c.min_inl) return;  // vFlow.cpp:934-942
    (void)dtdp;
    vx_out = r0;  // the plane's slopes: k_flow turns them into (Vx, Vy) (vFlow.cpp:1373-1377)
    vy_out = r1;
    acc_out = true;
}

// Variant that keeps the union: every lane writes the stamps of its union
// columns to the wave's LDS tile (ut[cell * kFitQS], cell = column * US + row) and
// their visited bits to a register mask, so the winning window needs no second
// round of loads (window column cxo is union column (bw / 3) * FR + cxo).
template <int FR>
__device__ __forceinline__ void fit_event_quad_u(const Ctx &c, int4 fd, uint32_t seq, int j, uint32_t *ut, double &vx_out,
                                                 double &vy_out, bool &acc_out) {
    (void)seq;
    constexpr int side = 2 * FR + 1, np = side * side, US = 4 * FR + 1;
    const int W = c.W, H = c.H;
    const int e = fd.x, ex = fd.y, ey = fd.z;  // the fit descriptor (k_fit_desc)
    const uint32_t te = (uint32_t)fd.w;
    vx_out = 0.0;
    vy_out = 0.0;
    acc_out = false;
    bool wok[9];
    int64_t score[9];
    bool any = false;
#pragma unroll
    for (int w = 0; w < 9; ++w) {
        const int ci = ex + (w / 3 - 1) * FR, cj = ey + (w % 3 - 1) * FR;
        wok[w] = ci - FR >= 0 && ci + FR <= W - 1 && cj - FR >= 0 && cj + FR <= H - 1;
        score[w] = 0;
        any |= wok[w];
    }
    if (!any) return;  // uniform over the quad
    // ---- window scores (vFlow.cpp:870-912), exact int64: this lane's union
    // columns.  A cell outside the stored region reads the buffer's guard head
    // (index WH: zero, never written), which resolves to "never visited", as
    // the reference's Event(0,0,0,0) cells do; cells outside the sensor also
    // read it and only enter the scores of windows the clip rejects (wok) and
    // union slots no accepted window reads, so they need no test of their own.
    uint64_t umask = 0;  // visited bits of this lane's union cells: (slot * US + row), slot = column / 4
    uint64_t pend = 0;   // cells whose tail decides (sae_head_stamp): fixed after the scan
    constexpr int NC = (US + 3) / 4;  // union columns per lane (the last one absent on some lanes)
    // t_e - t_k + [t_k > t_e] 2^32 (vFlow.cpp:891-905) is the 32-bit wrapped
    // difference, zero-extended: both lie in [0, 2^32) and agree mod 2^32
    auto ddiff = [&](uint32_t tk) { return (int64_t)(uint32_t)(te - tk); };
    const uint32_t guard = (uint32_t)c.WH;
#pragma unroll
    for (int sl = 0; sl < NC; ++sl) {  // unrolled: the loads of every column are in flight together
        const int du = -2 * FR + j + 4 * sl;
        if (du > 2 * FR) continue;
        const int u0 = ex + du, v0 = ey - 2 * FR;
        const bool inr = u0 >= c.X0 && u0 < c.XR1;  // (the stored region lies inside the sensor)
        const int cbase = (u0 - c.X0) * H + v0;
        uint3 col[US];
#pragma unroll
        for (int i = 0; i < US; ++i) {
            // unconditional loads (a load under a branch is waited for at the
            // branch's end, serializing the column)
            const bool ok = inr && v0 + i >= 0 && v0 + i < H;
            col[i] = sae_head(c, ok ? (uint32_t)(cbase + i) : guard);
        }
        const int ucol = du + 2 * FR;  // union column index
        int64_t dd[US];
#pragma unroll
        for (int i = 0; i < US; ++i) {
            bool vis, defer;
            const uint32_t tk = sae_head_stamp(col[i], e, vis, defer);
            ut[(ucol * US + i) * kFitQS] = tk;
            umask |= vis ? 1ull << (sl * US + i) : 0ull;
            pend |= defer ? 1ull << (sl * US + i) : 0ull;
            dd[i] = ddiff(tk);
        }
#pragma unroll
        for (int ovi = 0; ovi < 3; ++ovi) {
            int64_t sv = 0;
#pragma unroll
            for (int i = ovi * FR; i <= ovi * FR + 2 * FR; ++i) sv += dd[i];
#pragma unroll
            for (int oui = 0; oui < 3; ++oui) {
                const int ou = (oui - 1) * FR;
                if (du - ou <= FR && ou - du <= FR) score[oui * 3 + ovi] += sv;
            }
        }
    }
    // ---- the deferred cells: their tails, four loads in flight at a time;
    // each corrected stamp replaces the provisional t1 in the union tile and in
    // the scores of the windows that contain the cell (exact integers: any order)
#pragma unroll 1
    while (pend) {
        int bit[4];
        uint4 g[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            bit[k] = pend ? (int)__builtin_ctzll(pend) : -1;
            pend &= pend ? pend - 1 : 0ull;
            const int b = bit[k] < 0 ? 0 : bit[k];
            const int ucol = j + 4 * (b / US), i = b % US;
            const uint32_t q = (uint32_t)((ex + ucol - 2 * FR - c.X0) * H + ey + i - 2 * FR);
            g[k] = reinterpret_cast<const uint4 *>(c.cells.tail)[bit[k] < 0 ? 0u : q];  // e2m, t2, run_lo, run_hi
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (bit[k] < 0) continue;
            const int ucol = j + 4 * (bit[k] / US), i = bit[k] % US;
            uint32_t *slot = &ut[(ucol * US + i) * kFitQS];
            const uint32_t t1 = *slot;
            const uint32_t tk = sae_fix_tail(c, g[k], t1, e);
            if (tk == t1) continue;
            *slot = tk;
            const int64_t delta = ddiff(tk) - ddiff(t1);
            const int du = ucol - 2 * FR;
#pragma unroll
            for (int w = 0; w < 9; ++w) {
                const int ou = (w / 3 - 1) * FR, ovi = w % 3;
                if (du - ou <= FR && ou - du <= FR && i >= ovi * FR && i <= ovi * FR + 2 * FR) score[w] += delta;
            }
        }
    }
#pragma unroll
    for (int w = 0; w < 9; ++w) score[w] = quad_sum_i64(score[w]);
    const int64_t nn = np;
    int64_t best = nn * ((int64_t(1) << 32) + 1);  // MAXSTAMP + 1 per cell
    int bw = -1;
#pragma unroll
    for (int w = 0; w < 9; ++w)
        if (wok[w] && score[w] < best) { best = score[w]; bw = w; }
    if (bw < 0 || best > nn * (int64_t(1) << 32)) return;  // uniform over the quad

    // ---- the winning window, cx-major (vFlow.cpp:923-930), from the union tile:
    // visited bits of the window cells of this lane's columns, combined over the quad
    const int bi = ex + (bw / 3 - 1) * FR, bj = ey + (bw % 3 - 1) * FR;
    const int ub = (bw / 3) * FR, vb = (bw % 3) * FR;  // window origin in the union
    uint64_t vis = 0;
#pragma unroll
    for (int cxo = 0; cxo < side; ++cxo) {
        const int uc = ub + cxo;
        if ((uc & 3) != j) continue;
        const uint64_t colbits = (umask >> ((uc >> 2) * US + vb)) & ((1ull << side) - 1);
        vis |= colbits << (cxo * side);
    }
    vis = quad_or_u64(vis);
    // the union stamps were written by the other lanes of this wave's quad
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // This lane's window cells k = j, j + 4, ... (cx-major, k = kx * side + ky)
    // through a cursor advanced by 4 cells: the stored coordinates (a
    // never-visited cell stores (0, 0): vFlow.cpp:1226-1233) and the stamp in
    // the union tile (slot ofs = (ub + kx) * US + vb + ky)
    struct Cursor {
        int kx, ky, ofs;
        uint64_t vs;  // vis >> k
    };
    auto cursor = [&]() {
        Cursor q;
        q.kx = j / side;
        q.ky = j % side;
        q.ofs = (ub + q.kx) * US + vb + q.ky;
        q.vs = vis >> j;
        return q;
    };
    auto advance = [&](Cursor &q) {
        q.ky += 4;
        q.ofs += 4;
        q.vs >>= 4;
        if (q.ky >= side) { q.ky -= side; ++q.kx; q.ofs += US - side; }
        if constexpr (side < 5)
            if (q.ky >= side) { q.ky -= side; ++q.kx; q.ofs += US - side; }
    };
    auto cell = [&](const Cursor &q, uint32_t &X, uint32_t &Y, uint32_t &T) {
        const uint32_t m = 0u - (uint32_t)(q.vs & 1);  // all ones if visited
        X = (uint32_t)(bi + q.kx - FR) & m;
        Y = (uint32_t)(bj + q.ky - FR) & m;
        T = ut[q.ofs * kFitQS];
    };
    // Y (vFlow.cpp:1229-1233): t * 1e-6, or (t - 2^32) * 1e-6 for a stamp in the
    // event's future; t - 2^32 and t + 0 are exact in double, so adding the
    // selected offset before the one multiply is the reference's expression
    auto ytime = [&](uint32_t T) { return ((double)T + (T > te ? -kMaxStamp : 0.0)) * kTsToSec; };
    constexpr int NF = np / 4;  // full rounds of four cells (np % 4 == 1: one cell, lane 0's, after them)
    // AtA (vFlow.cpp:1307-1311): integer sums, exact in any split and order
    // (coordinates < 2^16: the 24-bit products are exact)
    int64_t sxx = 0, sxy = 0, sx = 0, syy = 0, sy = 0;
    {
        Cursor q = cursor();
#pragma unroll 1
        for (int it = 0; it <= NF; ++it) {
            uint32_t X, Y, T;
            cell(q, X, Y, T);
            if (it == NF && j != 0) X = Y = 0;  // past the window (adds nothing)
            sxx += __umul24(X, X); sxy += __umul24(X, Y); sx += X; syy += __umul24(Y, Y); sy += Y;
            advance(q);
        }
    }
    sxx = quad_sum_i64(sxx); sxy = quad_sum_i64(sxy); sx = quad_sum_i64(sx);
    syy = quad_sum_i64(syy); sy = quad_sum_i64(sy);
    const double a[9] = {(double)sxx, (double)sxy, (double)sx, (double)sxy, (double)syy,
                         (double)sy,  (double)sx,  (double)sy, (double)np};
    double DET = det3_partialpivlu(a);
    if (DET < 1) return;  // 0 inliers; uniform over the quad
    DET = 1.0 / DET;  // vFlow.cpp:1327-1336, A2 column-major
    const double d0 = DET * (a[8] * a[4] - a[7] * a[5]);
    const double d1 = DET * (a[7] * a[2] - a[8] * a[1]);
    const double d3 = DET * (a[6] * a[5] - a[8] * a[3]);
    const double d4 = DET * (a[8] * a[0] - a[6] * a[2]);
    const double d6 = DET * (a[7] * a[3] - a[6] * a[4]);  // (d2, d5, d8: the intercept row, never used)
    const double d7 = DET * (a[6] * a[1] - a[7] * a[0]);
    constexpr bool gemm = (3 + 3 + np) >= 20, gemv = (np + 3 + 1) >= 20;
    const double cz = (double)te * kTsToSec;
    // (A2 * At) * Y in the reference order (r2, the intercept, is never used:
    // vFlow.cpp:1352-1377).  Each term m_k * yt_k is one rounded product,
    // independent of the others, so lane j of the quad forms the terms of its
    // cells k = 4 it + j, and the sums then add them in order k = 0, 1, ... on
    // every lane (quad broadcasts): the additions are the reference's, a quarter
    // of the products per lane.
    auto terms = [&](const Cursor &q, double &q0, double &q1) {
        uint32_t Xi, Yi, T;
        cell(q, Xi, Yi, T);
        const double X = (double)Xi, Y = (double)Yi, yt = ytime(T);
        double m0, m1;
        if (gemm) {
            m0 = (((0.0 + d0 * X) + d3 * Y) + d6 * 1.0) + 0.0;
            m1 = (((0.0 + d1 * X) + d4 * Y) + d7 * 1.0) + 0.0;
        } else {
            m0 = (d0 * X + d3 * Y) + d6 * 1.0;
            m1 = (d1 * X + d4 * Y) + d7 * 1.0;
        }
        q0 = m0 * yt;
        q1 = m1 * yt;
    };
    double r0 = 0.0, r1 = 0.0;
    {
        Cursor q = cursor();
#pragma unroll 1
        for (int it = 0; it < NF; ++it) {
            double q0, q1;
            terms(q, q0, q1);
            const double a0 = quad_bcast<0>(q0), a1 = quad_bcast<0>(q1);
            if (!gemv && it == 0) { r0 = a0; r1 = a1; }
            else { r0 = r0 + a0; r1 = r1 + a1; }
            r0 = r0 + quad_bcast<1>(q0); r1 = r1 + quad_bcast<1>(q1);
            r0 = r0 + quad_bcast<2>(q0); r1 = r1 + quad_bcast<2>(q1);
            r0 = r0 + quad_bcast<3>(q0); r1 = r1 + quad_bcast<3>(q1);
            advance(q);
        }
        // the last cell, k = np - 1 = 4 NF: lane 0's (the other lanes' cursors
        // are past the window and read some slot of the union tile: unused)
        double q0, q1;
        terms(q, q0, q1);
        r0 = r0 + quad_bcast<0>(q0);
        r1 = r1 + quad_bcast<0>(q1);
    }
    if (gemv) { r0 = r0 + 0.0; r1 = r1 + 0.0; }
    const double dtdp = sqrt(r0 * r0 + r1 * r1);  // vFlow.cpp:1349-1377 (pow(v,2.0) as v*v)
    const double half = dtdp / 2;
    const double ccx = (double)ex, ccy = (double)ey;
    int inliers = 0;
    {
        Cursor q = cursor();
#pragma unroll 1
        for (int it = 0; it <= NF; ++it) {
            uint32_t Xi, Yi, T;
            cell(q, Xi, Yi, T);
            const double yt = ytime(T);
            const double planedt = (r0 * ((double)Xi - ccx) + r1 * ((double)Yi - ccy));
            const double actualdt = yt - cz;
            if (fabs(planedt - actualdt) < half && yt > 0 && (it < NF || j == 0)) ++inliers;
            advance(q);
        }
    }
    inliers += xch32<0>(inliers);
    inliers += xch32<1>(inliers);
    if (inliers < c.min_inl) return;  // vFlow.cpp:934-942
    vx_out = r0;  // the plane's slopes: k_flow turns them into (Vx, Vy) (vFlow.cpp:1373-1377)
    vy_out = r1;
    acc_out = true;
}

// Variant with rows per lane: lane j of the quad scans union rows j, j + 4, ...
// over every union column, so in each load instruction the quad's four lanes
// read four consecutive rows of one column -- consecutive x-major cells, one
// 64-B span of the SAE head array -- where the column mapping reads four cells
// a column (H cells) apart.  Scores, union tile and results as in
// fit_event_quad_u; the visited bits are kept row-major (bit (row slot) * US +
// column of the union, then cyo * side + cxo of the window).
template <int FR>
__device__ __forceinline__ void fit_event_quad_r(const Ctx &c, int4 fd, uint32_t seq, int j, uint32_t *ut, double &vx_out,
                                                 double &vy_out, bool &acc_out) {
    constexpr int side = 2 * FR + 1, np = side * side, US = 4 * FR + 1;
    constexpr int NR = (US + 3) / 4;  // union rows per lane (the last one absent on some lanes)
    static_assert(NR * US <= 64, "visited bits of a lane's union cells in one word");
    const int W = c.W, H = c.H;
    const int e = fd.x, ex = fd.y, ey = fd.z;  // the fit descriptor (k_fit_desc)
    const uint32_t te = (uint32_t)fd.w;
    vx_out = 0.0;
    vy_out = 0.0;
    acc_out = false;
    bool wok[9];
    int64_t score[9];
    bool any = false;
#pragma unroll
    for (int w = 0; w < 9; ++w) {
        const int ci = ex + (w / 3 - 1) * FR, cj = ey + (w % 3 - 1) * FR;
        wok[w] = ci - FR >= 0 && ci + FR <= W - 1 && cj - FR >= 0 && cj + FR <= H - 1;
        score[w] = 0;
        any |= wok[w];
    }
    if (!any) return;  // uniform over the quad
    // ---- window scores (vFlow.cpp:870-912), exact int64: this lane's union rows
    uint64_t umask = 0;  // visited bits: (row slot) * US + union column
    const int v0 = ey - 2 * FR;
#pragma unroll 1
    for (int cb = 0; cb < US; cb += 3) {  // three union columns at a time: their loads in flight together
        uint3 col[3][NR];
#pragma unroll
        for (int cc = 0; cc < 3; ++cc) {
            const int ucol = cb + cc;
            const int u = ex + ucol - 2 * FR;
            const bool inr = ucol < US && u >= 0 && u < W && u >= c.X0 && u < c.XR1;  // outside the stored region: never visited
            const int cbase = (u - c.X0) * H + v0;
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const int i = j + 4 * r, v = v0 + i;
                // unconditional load from a clamped index, then select (a load
                // under a branch is waited for at the branch end)
                const bool ok = inr && i < US && v >= 0 && v < H;
                const uint3 hd = sae_head(c, ok ? (uint32_t)(cbase + i) : 0u);
                col[cc][r] = ok ? hd : make_uint3(0, 0, 0);
            }
        }
#pragma unroll
        for (int cc = 0; cc < 3; ++cc) {
            const int ucol = cb + cc;
            const int u = ex + ucol - 2 * FR;
            if (ucol >= US || u < 0 || u >= W) continue;
            int64_t sv[3] = {0, 0, 0};  // this lane's part of the column sum of each window row range
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const int i = j + 4 * r, v = v0 + i;
                if (i >= US || v < 0 || v >= H) continue;
                const int64_t st = sae_resolve_h(c, col[cc][r], (uint32_t)((u - c.X0) * H + v), e, seq);
                const uint32_t tk = st < 0 ? 0u : (uint32_t)st;
                ut[(ucol * US + i) * kFitQS] = tk;
                umask |= st >= 0 ? 1ull << (r * US + ucol) : 0ull;
                const int64_t d = (int64_t)te - (int64_t)tk + (tk > te ? (int64_t(1) << 32) : 0);
#pragma unroll
                for (int ovi = 0; ovi < 3; ++ovi)
                    if (i >= ovi * FR && i <= ovi * FR + 2 * FR) sv[ovi] += d;
            }
            const int du = ucol - 2 * FR;
#pragma unroll
            for (int oui = 0; oui < 3; ++oui) {
                const int ou = (oui - 1) * FR;
                if (du - ou <= FR && ou - du <= FR) {
#pragma unroll
                    for (int ovi = 0; ovi < 3; ++ovi) score[oui * 3 + ovi] += sv[ovi];
                }
            }
        }
    }
#pragma unroll
    for (int w = 0; w < 9; ++w) score[w] = quad_sum_i64(score[w]);
    const int64_t nn = np;
    int64_t best = nn * ((int64_t(1) << 32) + 1);  // MAXSTAMP + 1 per cell
    int bw = -1;
#pragma unroll
    for (int w = 0; w < 9; ++w)
        if (wok[w] && score[w] < best) { best = score[w]; bw = w; }
    if (bw < 0 || best > nn * (int64_t(1) << 32)) return;  // uniform over the quad

    // ---- the winning window (vFlow.cpp:923-930) from the union tile: visited
    // bits of the window rows this lane holds (row-major, bit cyo * side +
    // cxo), combined over the quad
    const int bi = ex + (bw / 3 - 1) * FR, bj = ey + (bw % 3 - 1) * FR;
    const int ub = (bw / 3) * FR, vb = (bw % 3) * FR;  // window origin in the union
    uint64_t vis = 0;
#pragma unroll
    for (int cyo = 0; cyo < side; ++cyo) {
        const int ur = vb + cyo;
        if ((ur & 3) != j) continue;
        const uint64_t rowbits = (umask >> ((ur >> 2) * US + ub)) & ((1ull << side) - 1);
        vis |= rowbits << (cyo * side);
    }
    vis = quad_or_u64(vis);
    // the union stamps were written by the other lanes of this wave's quad
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    auto cell = [&](int k, int64_t &X, int64_t &Y, uint32_t &T) {  // k in the reference order: cx-major
        const int kx = k / side, ky = k % side;
        const int cx = bi + kx - FR, cy = bj + ky - FR;
        const bool vk = (vis >> (ky * side + kx)) & 1;
        X = vk ? cx : 0; Y = vk ? cy : 0; T = ut[((ub + kx) * US + vb + ky) * kFitQS];
    };
    int64_t sxx = 0, sxy = 0, sx = 0, syy = 0, sy = 0;  // exact: any split and order
#pragma unroll 1
    for (int k = j; k < np; k += 4) {
        int64_t X, Y; uint32_t T;
        cell(k, X, Y, T);
        sxx += X * X; sxy += X * Y; sx += X; syy += Y * Y; sy += Y;
    }
    sxx = quad_sum_i64(sxx); sxy = quad_sum_i64(sxy); sx = quad_sum_i64(sx);
    syy = quad_sum_i64(syy); sy = quad_sum_i64(sy);
    const double a[9] = {(double)sxx, (double)sxy, (double)sx, (double)sxy, (double)syy,
                         (double)sy,  (double)sx,  (double)sy, (double)np};
    double DET = det3_partialpivlu(a);
    if (DET < 1) return;  // 0 inliers; uniform over the quad
    DET = 1.0 / DET;  // vFlow.cpp:1327-1336, A2 column-major
    const double d0 = DET * (a[8] * a[4] - a[7] * a[5]);
    const double d1 = DET * (a[7] * a[2] - a[8] * a[1]);
    const double d3 = DET * (a[6] * a[5] - a[8] * a[3]);
    const double d4 = DET * (a[8] * a[0] - a[6] * a[2]);
    const double d6 = DET * (a[7] * a[3] - a[6] * a[4]);  // (d2, d5, d8: the intercept row, never used)
    const double d7 = DET * (a[6] * a[1] - a[7] * a[0]);
    constexpr bool gemm = (3 + 3 + np) >= 20, gemv = (np + 3 + 1) >= 20;
    const double cz = (double)te * kTsToSec;
    // (A2 * At) * Y in the reference order (r2, the intercept, is never used:
    // vFlow.cpp:1352-1377).  Each term m_k * yt_k is one rounded product,
    // independent of the others, so lane j of the quad forms the terms of
    // cells k = kb + j, and the sums then add them in order k = 0, 1, ... on
    // every lane (quad broadcasts): the additions are the reference's, a quarter
    // of the products per lane.
    double r0 = 0.0, r1 = 0.0;
#pragma unroll 1
    for (int kb = 0; kb < np; kb += 4) {
        const int k = kb + j < np ? kb + j : np - 1;
        int64_t Xi, Yi; uint32_t T;
        cell(k, Xi, Yi, T);
        const double X = (double)Xi, Y = (double)Yi, Tk = (double)T;
        const double yt = T > te ? (Tk - kMaxStamp) * kTsToSec : Tk * kTsToSec;
        double m0, m1;
        if (gemm) {
            m0 = (((0.0 + d0 * X) + d3 * Y) + d6 * 1.0) + 0.0;
            m1 = (((0.0 + d1 * X) + d4 * Y) + d7 * 1.0) + 0.0;
        } else {
            m0 = (d0 * X + d3 * Y) + d6 * 1.0;
            m1 = (d1 * X + d4 * Y) + d7 * 1.0;
        }
        const double q0 = m0 * yt, q1 = m1 * yt;
        const double a0 = quad_bcast<0>(q0), a1 = quad_bcast<0>(q1);
        if (!gemv && kb == 0) { r0 = a0; r1 = a1; }
        else { r0 = r0 + a0; r1 = r1 + a1; }
        if (kb + 1 < np) { r0 = r0 + quad_bcast<1>(q0); r1 = r1 + quad_bcast<1>(q1); }
        if (kb + 2 < np) { r0 = r0 + quad_bcast<2>(q0); r1 = r1 + quad_bcast<2>(q1); }
        if (kb + 3 < np) { r0 = r0 + quad_bcast<3>(q0); r1 = r1 + quad_bcast<3>(q1); }
    }
    if (gemv) { r0 = r0 + 0.0; r1 = r1 + 0.0; }
    const double dtdp = sqrt(r0 * r0 + r1 * r1);  // vFlow.cpp:1349-1377 (pow(v,2.0) as v*v)
    const double ccx = (double)ex, ccy = (double)ey;
    int inliers = 0;
#pragma unroll 1
    for (int k = j; k < np; k += 4) {
        int64_t Xi, Yi; uint32_t T;
        cell(k, Xi, Yi, T);
        const double Tk = (double)T;
        const double yt = T > te ? (Tk - kMaxStamp) * kTsToSec : Tk * kTsToSec;
        const double planedt = (r0 * ((double)Xi - ccx) + r1 * ((double)Yi - ccy));
        const double actualdt = yt - cz;
        if (fabs(planedt - actualdt) < dtdp / 2 && yt > 0) ++inliers;
    }
    inliers += xch32<0>(inliers);
    inliers += xch32<1>(inliers);
    if (inliers < c.min_inl) return;  // vFlow.cpp:934-942
    (void)dtdp;
    vx_out = r0;  // the plane's slopes: k_flow turns them into (Vx, Vy) (vFlow.cpp:1373-1377)
    vy_out = r1;
    acc_out = true;
}

// Four lanes per event of chunk [c0, c1) in tile order; lane 0 of the quad stores.
// (MODE 0: re-gather the winning window; 1: union tile, columns per lane;
// 2: union tile, rows per lane)
// Occupancy floor of the quad fit: fs <= 5 fits keep 7 waves per SIMD (at
// most 72 VGPRs; their 5.2-KB LDS tile allows 7.5); the fs-7 fit is held to
// 3.75 waves per SIMD by its 10.8-KB tile anyway, so it may use 128 VGPRs.
template <int FR>
constexpr int kFitMinWaves = FR <= 2 ? 7 : 1;
template <int FR, int MODE>
__global__ __launch_bounds__(64, kFitMinWaves<FR>) void k_fit_quad(Ctx c, int c0, int c1, uint32_t seq, FitPrep pr) {
    const int G = (int)gridDim.x - pr.blocks;  // the fit's blocks
    if ((int)blockIdx.x >= G) {
        fit_prep_thread(c, pr.cells, pr.p0, pr.c0, pr.c1, pr.seq,
                        ((int)blockIdx.x - G) * (int)blockDim.x + (int)threadIdx.x);
        return;
    }
    const int bid = (int)blockIdx.x;
#ifdef FARMS_FIT_VFLOOR  // tuning builds (make variant DEFS=-DFARMS_FIT_VFLOOR=\"v79\"): a VGPR floor for the fit
    asm volatile("" ::: FARMS_FIT_VFLOOR);
#endif
    constexpr int NPC = MODE ? (4 * FR + 1) * (4 * FR + 1) : (2 * FR + 1) * (2 * FR + 1);
    __shared__ uint32_t s_tk[NPC * kFitQS];
    // (an XCD-contiguous split of a 1,024-block fit launch measured 7% slower,
    // its per-XCD work being uneven; runs of 8 blocks per XCD keep the share even)
    const int fb = xcd_block_grouped(bid, G);
    const int w = c0 + ((fb * (int)blockDim.x + (int)threadIdx.x) >> 2);
    if (w >= c1) return;  // whole quads
    const int j = threadIdx.x & 3;
    const int4 fd = c.fdesc[w];  // {event, x, y, t}: one 16-B load (k_fit_desc)
    // halo columns: flows come from their owner (farms_import_flows); the whole quad
    if (!c.fit_all && (fd.y < c.fit_lo || fd.y >= c.fit_hi)) return;
    double vx, vy;
    bool acc;
    if constexpr (MODE == 2) fit_event_quad_r<FR>(c, fd, seq, j, s_tk + (threadIdx.x >> 2), vx, vy, acc);
    else if constexpr (MODE == 1) fit_event_quad_u<FR>(c, fd, seq, j, s_tk + (threadIdx.x >> 2), vx, vy, acc);
    else fit_event_quad<FR>(c, fd, seq, j, s_tk + (threadIdx.x >> 2), vx, vy, acc);
    if (j == 0) fit_plane(c, fd.x, vx, vy, acc);
}

// ---------------------------------------------------------------------------
// Wave-cooperative fit of one event (any fRad, every lookup complete): the
// lanes resolve the stamps of the union of the 9 candidate windows into LDS
// (these lookups are the latency: pixels with many in-chunk events need a run
// search) and reduce the integer window scores and normal-matrix sums; lane 0
// then runs the order-sensitive (A2*At)*Y accumulation from LDS.  Arithmetic
// is that of fit_event, so results are bitwise those of the per-thread path.
constexpr int kFitWaveCap = 1024;  // union-window cells staged per wave
constexpr int kFitWaveBlocks = 2048;  // fixed grid of k_fit_wave (4 waves per block)

__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) v += __shfl_xor(v, off, 64);
    return v;
}

__device__ void fit_wave_event(const Ctx &c, int e, uint32_t seq, uint32_t *s_t, uint8_t *s_v, int lane) {
    const int fr = c.fr, side = 2 * fr + 1, np = side * side, US = 4 * fr + 1, nU = US * US;
    const int W = c.W, H = c.H;
    const int ex = c.x[e], ey = c.y[e];
    const uint32_t te = c.t[e];
    if (nU > kFitWaveCap) {  // very large filters: per-thread path on lane 0
        if (lane == 0) {
            double vx, vy;
            bool acc;
            fit_event_generic(c, e, seq, vx, vy, acc);
            fit_plane(c, e, vx, vy, acc);
        }
        return;
    }
    bool wok[9];
    bool any = false;
#pragma unroll
    for (int w = 0; w < 9; ++w) {
        const int ci = ex + (w / 3 - 1) * fr, cj = ey + (w % 3 - 1) * fr;
        wok[w] = ci - fr >= 0 && ci + fr <= W - 1 && cj - fr >= 0 && cj + fr <= H - 1;
        any |= wok[w];
    }
    if (!any) {
        if (lane == 0) fit_plane(c, e, 0.0, 0.0, false);
        return;
    }
    // ---- stage the union window and score the 9 windows (vFlow.cpp:870-912)
    int64_t score[9];
#pragma unroll
    for (int w = 0; w < 9; ++w) score[w] = 0;
    for (int idx = lane; idx < nU; idx += 64) {
        const int du = idx / US - 2 * fr, dv = idx % US - 2 * fr;
        const int u = ex + du, v = ey + dv;
        const bool ins = u >= 0 && u < W && v >= 0 && v < H;
        int64_t st = -1;
        if (ins && u >= c.X0 && u < c.XR1) st = sae_asof(c, (uint32_t)((u - c.X0) * H + v), e, seq);
        const uint32_t tk = st < 0 ? 0u : (uint32_t)st;
        s_t[idx] = tk;
        s_v[idx] = st >= 0 ? 1 : 0;
        if (ins) {
            const int64_t d = (int64_t)te - (int64_t)tk + (tk > te ? (int64_t(1) << 32) : 0);
#pragma unroll
            for (int w = 0; w < 9; ++w) {
                const int ou = (w / 3 - 1) * fr, ov = (w % 3 - 1) * fr;
                if (wok[w] && du - ou <= fr && ou - du <= fr && dv - ov <= fr && ov - dv <= fr) score[w] += d;
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const int64_t nn = np;
    int64_t best = nn * ((int64_t(1) << 32) + 1);
    int bw = -1;
#pragma unroll
    for (int w = 0; w < 9; ++w) {
        const int64_t sw = wave_sum_i64(score[w]);
        if (wok[w] && sw < best) { best = sw; bw = w; }
    }
    if (bw < 0 || best > nn * (int64_t(1) << 32)) {
        if (lane == 0) fit_plane(c, e, 0.0, 0.0, false);
        return;
    }
    // ---- the winning window, cx-major (vFlow.cpp:923-930)
    const int bi = ex + (bw / 3 - 1) * fr, bj = ey + (bw % 3 - 1) * fr;
    auto cell = [&](int k, int64_t &X, int64_t &Y, uint32_t &T) {
        const int cx = bi + k / side - fr, cy = bj + k % side - fr;
        const int idx = (cx - ex + 2 * fr) * US + (cy - ey + 2 * fr);
        const bool vk = s_v[idx] != 0;
        X = vk ? cx : 0; Y = vk ? cy : 0; T = s_t[idx];
    };
    int64_t sxx = 0, sxy = 0, sx = 0, syy = 0, sy = 0;
    for (int k = lane; k < np; k += 64) {
        int64_t X, Y; uint32_t T;
        cell(k, X, Y, T);
        sxx += X * X; sxy += X * Y; sx += X; syy += Y * Y; sy += Y;
    }
    sxx = wave_sum_i64(sxx); sxy = wave_sum_i64(sxy); sx = wave_sum_i64(sx);
    syy = wave_sum_i64(syy); sy = wave_sum_i64(sy);
    const double a[9] = {(double)sxx, (double)sxy, (double)sx, (double)sxy, (double)syy,
                         (double)sy,  (double)sx,  (double)sy, (double)np};
    double DET = det3_partialpivlu(a);
    int inliers = 0;
    double dtdx = 0.0, dtdy = 0.0;
    if (!(DET < 1)) {
        DET = 1.0 / DET;  // vFlow.cpp:1327-1336
        const double d0 = DET * (a[8] * a[4] - a[7] * a[5]);
        const double d1 = DET * (a[7] * a[2] - a[8] * a[1]);
        const double d2 = DET * (a[5] * a[1] - a[4] * a[2]);
        const double d3 = DET * (a[6] * a[5] - a[8] * a[3]);
        const double d4 = DET * (a[8] * a[0] - a[6] * a[2]);
        const double d5 = DET * (a[3] * a[2] - a[5] * a[0]);
        const double d6 = DET * (a[7] * a[3] - a[6] * a[4]);
        const double d7 = DET * (a[6] * a[1] - a[7] * a[0]);
        const double d8 = DET * (a[4] * a[0] - a[3] * a[1]);
        const bool gemm = (3 + 3 + np) >= 20, gemv = (np + 3 + 1) >= 20;
        const double cz = (double)te * kTsToSec;
        double r0 = 0.0, r1 = 0.0, r2 = 0.0;
        if (lane == 0) {  // order-sensitive: one lane, stamps from LDS
            for (int k = 0; k < np; ++k) {
                int64_t Xi, Yi; uint32_t T;
                cell(k, Xi, Yi, T);
                const double X = (double)Xi, Y = (double)Yi, Tk = (double)T;
                const double yt = T > te ? (Tk - kMaxStamp) * kTsToSec : Tk * kTsToSec;
                double m0, m1, m2;
                if (gemm) {
                    m0 = (((0.0 + d0 * X) + d3 * Y) + d6 * 1.0) + 0.0;
                    m1 = (((0.0 + d1 * X) + d4 * Y) + d7 * 1.0) + 0.0;
                    m2 = (((0.0 + d2 * X) + d5 * Y) + d8 * 1.0) + 0.0;
                } else {
                    m0 = (d0 * X + d3 * Y) + d6 * 1.0;
                    m1 = (d1 * X + d4 * Y) + d7 * 1.0;
                    m2 = (d2 * X + d5 * Y) + d8 * 1.0;
                }
                if (!gemv && k == 0) { r0 = m0 * yt; r1 = m1 * yt; r2 = m2 * yt; }
                else { r0 = r0 + m0 * yt; r1 = r1 + m1 * yt; r2 = r2 + m2 * yt; }
            }
            if (gemv) { r0 = r0 + 0.0; r1 = r1 + 0.0; r2 = r2 + 0.0; }
        }
        r0 = __shfl(r0, 0, 64);
        r1 = __shfl(r1, 0, 64);
        const double dtdp = sqrt(r0 * r0 + r1 * r1);
        const double ccx = (double)ex, ccy = (double)ey;
        int inl = 0;
        for (int k = lane; k < np; k += 64) {
            int64_t Xi, Yi; uint32_t T;
            cell(k, Xi, Yi, T);
            const double Tk = (double)T;
            const double yt = T > te ? (Tk - kMaxStamp) * kTsToSec : Tk * kTsToSec;
            const double planedt = (r0 * ((double)Xi - ccx) + r1 * ((double)Yi - ccy));
            const double actualdt = yt - cz;
            if (fabs(planedt - actualdt) < dtdp / 2 && yt > 0) ++inl;
        }
        inliers = (int)wave_sum_i64(inl);
        dtdx = r0;
        dtdy = r1;
    }
    if (lane == 0) {
        const bool acc = inliers >= c.min_inl;  // vFlow.cpp:934-942
        fit_plane(c, e, acc ? dtdx : 0.0, acc ? dtdy : 0.0, acc);
    }
}

// Waves loop over the events list[0 .. count) (every event of a chunk, for
// filters without a compile-time fast path).  The grid is fixed; every wave
// reaches the loop end.
__global__ __launch_bounds__(256) void k_fit_wave(Ctx c, uint32_t seq, const int32_t *list, int count) {
    __shared__ uint32_t s_t[4][kFitWaveCap];
    __shared__ uint8_t s_v[4][kFitWaveCap];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int n = count;
    const int stride = (int)gridDim.x * 4;
    for (int i = (int)blockIdx.x * 4 + wv; i < n; i += stride) {
        if (!c.fit_all) {
            const int ex = c.x[list[i]];
            if (ex < c.fit_lo || ex >= c.fit_hi) continue;  // wave-uniform
        }
        fit_wave_event(c, list[i], seq, s_t[wv], s_v[wv], lane);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

// cells per candidate group = one k_chain wavefront (4 bitmap words).  Measured
// at C3 (round 3): 128 cells (78 VGPRs, 6 waves; or 64 VGPRs, 8 waves) 92-95 ms
// per step, 512 cells (229 VGPRs, 2 waves) 95 ms, against 87.5 for 256: more
// chain waves take slots from the fit and pooling, fewer lengthen the chain.
// acc + the set bits of m below this lane (v_mbcnt_lo / v_mbcnt_hi: two VALU
// in place of a mask, two ANDs and two bit counts)
__device__ __forceinline__ int mbcnt64(uint64_t m, int acc) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, (uint32_t)acc));
}

// Inclusive prefix sum over the 64 lanes with DPP: row shifts inside each
// 16-lane row, then the row broadcasts of lanes 15 and 31.
__device__ __forceinline__ int wave_incl_scan(int v) {
    // (as half_incl_scan, then row_bcast:31 into rows 2 and 3)
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, true);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, true);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, true);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, true);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return v;
}

constexpr int kGroupCells = 256;

// The call's candidate-build plan (Ctx::cinfo, per workspace set):
//   kCiMaxBack  largest chunk distance back to cbk (k_cand_plan_back)
//   kCiCount    call-start snapshot list length (k_cand_list)
//   kCiLMin/Max stamp range of that list
//   kCiTMin/Max stamp range of the call's events
enum { kCiMaxBack = 0, kCiCount, kCiLMin, kCiLMax, kCiTMin, kCiTMax, kCiWords };
// k_cand takes a call when every chunk's kill window reaches back at most this
// many chunks (a time-ordered stream: 2-3); other streams (out-of-order stamps)
// keep k_chain, whose cost is independent of the order.  The host reads the
// reach after the call's prep (k_cand_plan_back) and launches one of the two.
constexpr int kCandMaxBack = 64;
constexpr int kPoisonByte = 0x7F;  // FARMS_POISON's fill (farms_handle::poison)


// The pooling sweep's candidate chain, one launch per super-chunk (pooling
// chunks [ch0, ch1)).  A wavefront owns one candidate group (kGroupCells = 256
// cells = 4 bitmap words, lane = cell of each word); the group's candidates of
// a chunk take slots [g * 256, ...) of the chunk's ring buffer, so the word
// offsets are a scalar prefix of the wave's 4 ballots — no block barrier, no
// global scan, and the waves of a launch never wait for each other.  Each
// cell's state stays in registers across the chunks: the cursor into its run
// of P (next event id nxt), its flow snapshot (snap; ft = its stamp, -1 when
// the snapshot flow is invalid), and, prefetched one touch ahead, the local
// flow of the next event at the cell and the run entry after it (pf, pnx), so
// a chunk's common case (one event at the cell) issues no dependent load.
// Per chunk ch (ring buffer ch % NB):
//   bit(q) = q's snapshot flow is valid and its stamp within the kill time
//            of the chunk's stamp span, or q's first event in ch has valid
//            flow, or q fires more than once in ch: a superset of every cell
//            that can contribute to an event of ch as of that event
//            (vFlow.cpp:1002/1115);
//   bitmap words + group-local candidate offsets;
//   fill: candidate record = snapshot flow before ch + first in-chunk flow
//         and the cell's in-chunk run bounds in P;
//   advance: snapshot <- last in-chunk event at q, cursor past the chunk,
//            prefetch of the next touch (events of the super-chunk only: the
//            fit of later events may still be running).
// The state round-trips memory once per launch (only cells touched in it).
constexpr int kChainCells = kGroupCells / 64;  // cells per lane
struct ChainFlow {  // FlowCell without its padding: L, L cos, L sin, stamp
    double L, Lc, Ls;
    uint32_t t;
};
__device__ __forceinline__ ChainFlow chain_load(const FlowCell *p) {
    const FlowCell f = *p;
    return ChainFlow{f.L, f.Lc, f.Ls, f.t};
}
// One-wave workgroups (a 4-wave one needs 4 x 128 VGPRs free at once on one
// CU, which the pooling waves rarely leave), at most 128 VGPRs (4 waves per SIMD).
#ifndef FARMS_CHAIN_WAVES  // tuning builds: k_chain's minimum waves per SIMD (VGPR budget)
#define FARMS_CHAIN_WAVES 4
#endif
__global__ __launch_bounds__(64, FARMS_CHAIN_WAVES) void k_chain(Ctx c, int ch0, int ch1) {
    const int lane = threadIdx.x & 63;
    const int64_t g = (int64_t)blockIdx.x;
    if (g >= c.nblk) return;
    const int n = c.n, C2 = c.C2;
    const int lim = min(ch1 * C2, n);  // local flows of events < lim are final
    int k[kChainCells], kend[kChainCells], nxt[kChainCells], pnx[kChainCells];
    ChainFlow snap[kChainCells], pf[kChainCells];
    uint32_t dirty = 0;
    // the next touch of cell i: its flow and the run entry after it, loaded
    // when the cell moves.  (Round 4 tried loading them for every lane and cell
    // slot after each chunk from clamped indices, so that no load sat under a
    // branch: the untouched cells' loads all went to evf[0] and P[0], one L2
    // channel, and a C3 step took 184 ms against 89.)
    auto prefetch = [&](int i) {
        pnx[i] = INT_MAX;
        pf[i] = ChainFlow{0.0, 0.0, 0.0, 0u};
        if (nxt[i] < lim) {
            pf[i] = chain_load(&c.evf[nxt[i]]);
            if (k[i] + 1 <= kend[i]) pnx[i] = c.P[k[i] + 1];
        }
    };
    auto pnext = [&](int i) { return pnx[i]; };
#pragma unroll
    for (int i = 0; i < kChainCells; ++i) {
        const int64_t q = (g * kChainCells + i) * 64 + lane;
        k[i] = 0; kend[i] = -1;
        int64_t ft = -1;
        if (q < c.WH) {
            kend[i] = c.pend[q];
            if (kend[i] >= 0) k[i] = c.pcur[q];  // pcur is only defined for cells with events in this call
            ft = c.ftime[q];
        }
        nxt[i] = k[i] <= kend[i] ? c.P[k[i]] : INT_MAX;
        snap[i] = ChainFlow{0.0, 0.0, 0.0, 0u};  // an invalid snapshot flow is never read (kCandSnapOk clear)
        if (ft >= 0) snap[i] = chain_load(&c.fsnap[q]);
    }
#pragma unroll
    for (int i = 0; i < kChainCells; ++i) prefetch(i);
    // the chunks' stamp spans, lane l holding chunk ch0 + l (read with a
    // wave-uniform readlane: no memory round trip per chunk; a launch covers
    // at most 64 chunks).  Unconditional loads from a clamped index: a
    // conditional one merged into the same register would make every readlane
    // wait for all outstanding loads, the prefetches included.
    const int chl = min(ch0 + lane, ch1 - 1);
    const uint32_t tmin_l = c.ctmin[chl];
    const uint32_t tmax_l = c.ctmax[chl];
    // wait for them here, once
    asm volatile("" ::"v"(tmin_l), "v"(tmax_l));
    for (int ch = ch0; ch < ch1; ++ch) {
        const int b = (c.ring0 + ch) % c.NB;
        const int ce = min((ch + 1) * C2, n);
        const uint32_t tmin = (uint32_t)__builtin_amdgcn_readlane((int)tmin_l, ch - ch0);
        const uint32_t tmax = (uint32_t)__builtin_amdgcn_readlane((int)tmax_l, ch - ch0);
        const int64_t lo = (int64_t)tmin - (int64_t)kKillUs, hi = (int64_t)tmax + (int64_t)kKillUs;
        uint64_t bal[kChainCells];
        uint32_t woff[kChainCells];
        uint32_t acc = (uint32_t)(g * kGroupCells);
#pragma unroll
        for (int i = 0; i < kChainCells; ++i) {
            // a candidate can contribute to some event of the chunk: through its
            // snapshot (valid flow, stamp within the kill time of the chunk's
            // span), or through an in-chunk event with valid flow (the first
            // one, or any of a longer run)
            const int64_t ts = (int64_t)snap[i].t;
            const bool bit = (snap[i].L > 0 && ts > lo && ts < hi) ||
                             (nxt[i] < ce && (pf[i].L > 0 || pnext(i) < ce));
            bal[i] = __ballot(bit);
            woff[i] = acc;
            acc += (uint32_t)__popcll(bal[i]);
            const int64_t w = g * kChainCells + i;
            if (lane == 0 && w < c.nwords) {
                BmWord *bw = c.bw_ring + (int64_t)b * c.nwords + w;
                bw->bm = bal[i];
                bw->wo = woff[i];
            }
        }
#pragma unroll
        for (int i = 0; i < kChainCells; ++i) {
            const int64_t q = (g * kChainCells + i) * 64 + lane;
            const bool touched = nxt[i] < ce;
            const int k1 = k[i];
            const int e1 = touched ? nxt[i] : INT_MAX;
            // one walk over the cell's in-chunk run (a longer run is rare): its last
            // position and event, and the run entry after the chunk
            int run_hi = k1, last = e1, nn = pnext(i);
            if (touched) {
                while (nn < ce) {
                    ++run_hi;
                    last = nn;
                    nn = run_hi + 1 <= kend[i] ? c.P[run_hi + 1] : INT_MAX;
                }
            }
            // the last in-chunk event's flow: the next snapshot, and (a run of two)
            // the second event inlined in the candidate record
            const ChainFlow fl = touched && last != e1 ? chain_load(&c.evf[last]) : pf[i];
            if ((bal[i] >> lane) & 1) {  // candidate record: snapshot before ch, first in-chunk flow, run bounds
                CandHdr hd;
                CandVal v;
                hd.lin = (uint32_t)q | (snap[i].L > 0 ? kCandSnapOk : 0u);
                hd.t_snap = snap[i].t;
                v.L_snap = snap[i].L; v.Lc_snap = snap[i].Lc; v.Ls_snap = snap[i].Ls;
                if (touched) {
                    hd.e1 = e1;
                    hd.lin |= (run_hi > k1 ? kCandMore : 0u) | (run_hi > k1 + 1 ? kCandMore2 : 0u) |
                              (pf[i].L > 0 ? kCandOneOk : 0u);
                    hd.t1 = pf[i].t;
                    v.L1 = pf[i].L; v.Lc1 = pf[i].Lc; v.Ls1 = pf[i].Ls;
                    if (run_hi == k1 + 1) {  // two events: the second inline
                        v.run_lo = (int32_t)((uint32_t)last | (fl.L > 0 ? 0x80000000u : 0u));
                        v.run_hi = (int32_t)fl.t;
                    } else {
                        v.run_lo = k1; v.run_hi = run_hi;
                    }
                } else {
                    hd.e1 = INT_MAX;
                    hd.t1 = 0;
                    v.L1 = 0.0; v.Lc1 = 0.0; v.Ls1 = 0.0;
                    v.run_lo = 0; v.run_hi = 0;
                }
                const int64_t kb = (int64_t)b * c.cstride + (uint32_t)mbcnt64(bal[i], (int)woff[i]);
                c.hdr_ring[kb] = hd;
                c.val_ring[kb] = v;
            }
            if (touched) {  // advance: snapshot <- last event of the chunk at q; prefetch the next touch
                snap[i] = fl;
                k[i] = run_hi + 1;
                nxt[i] = nn;
                dirty |= 1u << i;
                prefetch(i);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < kChainCells; ++i) {
        const int64_t q = (g * kChainCells + i) * 64 + lane;
        if ((dirty >> i) & 1) {
            FlowCell f;
            f.L = snap[i].L; f.Lc = snap[i].Lc; f.Ls = snap[i].Ls; f.t = snap[i].t; f.pad = 0;
            c.fsnap[q] = f;
            c.ftime[q] = snap[i].L > 0 ? (int64_t)snap[i].t : -1;
            c.pcur[q] = k[i];
        }
    }
}

// ---------------------------------------------------------------------------
// Event-driven candidate build (k_cand): the same candidate lists as k_chain,
// from the events instead of a sweep over every cell.  k_chain keeps each
// cell's state in registers across a super-chunk's 64 chunks, one wave per
// 256 cells for the whole launch: 3,600 waves of 128 VGPRs at 1280 x 720,
// mostly waiting on one dependent round trip per chunk, while ~31% of the
// cells fire in a super-chunk and ~2% are candidates of a chunk.  Here the
// candidates of chunk ch = [cs, ce) come from three disjoint sources:
//   S1  the first event e at each cell touched in ch (link prev < cs): its
//       snapshot is the flow of the previous event at the cell (link prev),
//       or the call-start snapshot fsnap when the call had none;
//   S2  an earlier event e' of the call that is the last at its cell before ce
//       (link next >= ce) with valid flow and stamp inside the chunk's kill
//       window -- only chunks [cbk[ch], ch) can hold one (cbk from the prefix
//       maximum of the chunks' last stamps);
//   S3  a cell of the call-start snapshot list (valid snapshot flow) whose
//       stamp is inside the kill window and whose first event of the call is
//       at or past ce.
// bit(q) is k_chain's: S1 cells when the cell fires more than once in ch, its
// first flow is valid, or its snapshot is valid and inside the window; S2/S3
// cells always.  So the bitmap words and the records are k_chain's, the
// candidate slot of a cell is its rank in cell order inside its group, and
// k_pool reads the same lists.  Chunks are independent: one workgroup per
// (chunk, slice of the sensor's groups) marks its cells in an LDS bitmap,
// writes the words with their group-local offsets, then the records.
// fsnap holds the call-start snapshots while the call runs; k_cand_commit
// advances it to each cell's last event once the call's lists are built.

// Prefix maximum of the chunks' last stamps and the call's stamp span (one block).
__global__ __launch_bounds__(1024) void k_cand_plan_max(const uint32_t *tmin, const uint32_t *tmax, int nch,
                                                        uint32_t *pmax, int *info) {
    __shared__ uint32_t smax[1024], smin[1024];
    const int T = (int)blockDim.x, tid = (int)threadIdx.x;
    const int per = (nch + T - 1) / T;
    const int a = min(tid * per, nch), b = min(a + per, nch);
    uint32_t m = 0, mn = 0xFFFFFFFFu;
    for (int i = a; i < b; ++i) {
        m = max(m, tmax[i]);
        mn = min(mn, tmin[i]);
    }
    smax[tid] = m;
    smin[tid] = mn;
    __syncthreads();
    for (int off = 1; off < T; off <<= 1) {  // inclusive max-scan over the threads' segments
        const uint32_t v = tid >= off ? smax[tid - off] : 0u;
        __syncthreads();
        smax[tid] = max(smax[tid], v);
        __syncthreads();
    }
    uint32_t run = tid > 0 ? smax[tid - 1] : 0u;
    for (int i = a; i < b; ++i) {
        run = max(run, tmax[i]);
        pmax[i] = run;
    }
    for (int s = T / 2; s > 0; s >>= 1) {
        if (tid < s) smin[tid] = min(smin[tid], smin[tid + s]);
        __syncthreads();
    }
    if (tid == 0) {
        info[kCiMaxBack] = 0;
        info[kCiCount] = 0;
        info[kCiLMin] = (int)0xFFFFFFFFu;
        info[kCiLMax] = 0;
        info[kCiTMin] = (int)smin[0];
        info[kCiTMax] = (int)smax[T - 1];
    }
}

// cbk[ch]: the first chunk c' < ch whose prefix-maximum last stamp is inside
// ch's kill window (no event of an earlier chunk can be a snapshot candidate
// of ch: its stamp is <= tmin - 500); ch if none.
__global__ void k_cand_plan_back(const uint32_t *tmin, const uint32_t *pmax, int nch, int32_t *bk, int *info) {
    const int ch = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (ch >= nch) return;
    const int64_t lo = (int64_t)tmin[ch] - (int64_t)kKillUs;
    int a = 0, b = ch;
    while (a < b) {
        const int m = (a + b) >> 1;
        if ((int64_t)pmax[m] > lo) b = m;
        else a = m + 1;
    }
    bk[ch] = a;
    atomicMax(&info[kCiMaxBack], ch - a);
}

// The call-start snapshot list: cells whose snapshot flow is valid with a stamp
// inside the call's span widened by the kill time, with the first event of the
// call at the cell (INT_MAX: none).  Any order (k_cand's bitmap ranks them).
__global__ void k_cand_list(Ctx c, int4 *list) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int *info = c.cinfo;
    const int lane = (int)(threadIdx.x & 63);
    bool keep = false;
    int4 ent = make_int4(0, 0, 0, 0);
    if (q < c.WH) {
        const int64_t ft = c.ftime[q];
        const int64_t lo = (int64_t)(uint32_t)info[kCiTMin] - (int64_t)kKillUs,
                      hi = (int64_t)(uint32_t)info[kCiTMax] + (int64_t)kKillUs;
        if (ft >= 0 && ft > lo && ft < hi) {
            keep = true;
            const int first = c.pend[q] >= 0 ? c.P[c.pcur[q]] : INT_MAX;
            ent = make_int4((int)q, (int)(uint32_t)ft, first, 0);
        }
    }
    const uint64_t bal = __ballot(keep);
    if (!bal) return;
    const int leader = __ffsll((unsigned long long)bal) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(&info[kCiCount], (int)__popcll(bal));
    base = __shfl(base, leader, 64);
    if (keep) {
        const int i = base + (int)__popcll(bal & ((1ull << lane) - 1));
        list[i] = ent;
        atomicMin(reinterpret_cast<unsigned int *>(&info[kCiLMin]), (unsigned int)ent.y);
        atomicMax(reinterpret_cast<unsigned int *>(&info[kCiLMax]), (unsigned int)ent.y);
    }
}

// The work order of one pooling chunk per workgroup (round 4): its events'
// 8x8-tile keys sorted in LDS by a block radix sort (stable, so events of a
// tile stay in index order: the same Q as the device-wide sort of (chunk, tile)
// keys), and in the same pass the fit descriptors {event, x, y, t} (gathers
// inside the chunk's window), the column bands' work-order starts (k_cand)
// and the chunk's stamp span.  Replaces the second device-wide radix sort,
// k_fit_desc, k_band_starts and k_chunk_minmax for pooling chunks of 2,048,
// 4,096 and 8,192 events (C3 77.6-77.8 -> 77.2 ms per step,
// profiles/r04_ab_chunk_order.log).
// The events' fields are read and the work order / descriptors written in
// striped order (lane-consecutive ranks: coalesced); the blocked arrangement
// the stable sort takes is made through LDS on both sides (round 6: C3 67.1 ->
// 66.1 ms, profiles/r06_ab_chunk_order_striped_c3.log; the blocked reads and
// writes touched a 32-B-strided line per lane).
template <int THREADS, int ITEMS>
__global__ __launch_bounds__(THREADS) void k_chunk_order(Ctx c, int tile_bits, int32_t *Q, int32_t *bstart,
                                                         uint32_t *tmin, uint32_t *tmax) {
    using BRS = hipcub::BlockRadixSort<uint32_t, THREADS, ITEMS, int>;
    constexpr int N = THREADS * ITEMS;
    __shared__ union {
        typename BRS::TempStorage sort;
        uint32_t key[N];
        uint2 kv[N];
    } s_u;
    __shared__ uint32_t s_lo[THREADS / 64], s_hi[THREADS / 64];
    const int ch = (int)blockIdx.x, tid = (int)threadIdx.x;
    const int cs = ch * c.C2, cnt = min(c.C2, c.n - cs);
    const uint32_t pad = 1u << tile_bits;
    uint32_t lo = 0xFFFFFFFFu, hi = 0u;
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {  // striped: rank i * THREADS + tid
        const int r = i * THREADS + tid;
        uint32_t k = pad;
        if (r < cnt) {
            const int e = cs + r;
            const int x = c.x[e], y = c.y[e];
            const uint32_t t = c.t[e];
            k = (uint32_t)((x - c.X0) >> c.tshift) * (uint32_t)c.tilesH + (uint32_t)(y >> c.tshift);
            lo = t < lo ? t : lo;
            hi = t > hi ? t : hi;
        }
        s_u.key[r] = k;
    }
    __syncthreads();
    uint32_t key[ITEMS];
    int val[ITEMS];
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {  // blocked: rank tid * ITEMS + i (the stable sort's input order)
        key[i] = s_u.key[tid * ITEMS + i];
        val[i] = tid * ITEMS + i;
    }
    __syncthreads();
    BRS(s_u.sort).Sort(key, val, 0, tile_bits + 1);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) s_u.kv[tid * ITEMS + i] = make_uint2(key[i], (uint32_t)val[i]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        lo = min(lo, (uint32_t)__shfl_xor((int)lo, o, 64));
        hi = max(hi, (uint32_t)__shfl_xor((int)hi, o, 64));
    }
    if ((tid & 63) == 0) { s_lo[tid >> 6] = lo; s_hi[tid >> 6] = hi; }
    __syncthreads();
    const int tpb = c.bandc >> c.tshift;  // tile columns per band
    auto band = [&](uint32_t k) { return k >= pad ? c.nbands : (int)(k / (uint32_t)c.tilesH) / tpb; };
    int32_t *bs = bstart + (int64_t)ch * (c.nbands + 1);
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {  // striped again: coalesced Q / descriptor writes
        const int r = i * THREADS + tid;
        const uint2 kv = s_u.kv[r];
        const int b = band(kv.x);
        const int prev = r > 0 ? band(s_u.kv[r - 1].x) : -1;
        // the first rank of each band (padding ranks have band nbands: its start is cnt)
        for (int q = prev + 1; q <= b; ++q) bs[q] = cs + min(r, cnt);
        if (r == N - 1)  // bands past the last key (no padding when the chunk is full)
            for (int q = b + 1; q <= c.nbands; ++q) bs[q] = cs + cnt;
        if (r < cnt) {
            const int e = cs + (int)kv.y;
            Q[cs + r] = e;
            c.fdesc[cs + r] = make_int4(e, c.x[e], c.y[e], (int)c.t[e]);
        }
    }
    if (tid == 0) {
        uint32_t a = s_lo[0], b = s_hi[0];
        for (int u = 1; u < THREADS / 64; ++u) { a = min(a, s_lo[u]); b = max(b, s_hi[u]); }
        tmin[ch] = a;
        tmax[ch] = b;
    }
}

// Work-order bounds of the column bands (k_cand): the work order Q is sorted by
// (pooling chunk, 8x8 tile), tiles x-major, so the events of chunk ch in the
// band of columns [b * bandc, (b + 1) * bandc) are the positions
// [bstart[ch * (nbands + 1) + b], bstart[ch * (nbands + 1) + b + 1]).
__global__ void k_band_starts(Ctx c, const uint32_t *wkey_sorted, int tile_bits, int32_t *bstart) {
    const int w = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (w >= c.n) return;
    const int ch = w / c.C2, cs = ch * c.C2, ce = min(cs + c.C2, c.n);
    const uint32_t tmask = (1u << tile_bits) - 1;
    const int tpb = c.bandc >> c.tshift;  // tile columns per band
    auto band = [&](int i) { return (int)((wkey_sorted[i] & tmask) / (uint32_t)c.tilesH) / tpb; };
    const int bw = band(w), pb = w > cs ? band(w - 1) : -1;
    int32_t *bs = bstart + (int64_t)ch * (c.nbands + 1);
    for (int b = pb + 1; b <= bw; ++b) bs[b] = w;
    if (w == ce - 1)
        for (int b = bw + 1; b <= c.nbands; ++b) bs[b] = ce;
}

// k_cand's S2 sources of pooling chunks [ch0, ch1) (round 5): an event of
// chunk cp can be an S2 candidate of a later chunk ch only if it is the last
// event at its cell before ch's end -- so the last at its cell in cp (next
// event at or past cp's end) -- and its flow is valid.  One wavefront per
// (chunk, column band), as k_cand: the band's such events, compacted in work
// order to the front of the band's own work-order range {event, cell, stamp,
// next event}, and their number.  A later chunk's S2 then reads 16 B per such
// event of its band, where it read every event's descriptor, link and flow of
// each of the ~3 chunks its kill window reaches.  Runs on the chain stream
// after the super-chunk's flows (k_flow; the imports of an x-strip call) and
// before its k_cand.
__global__ __launch_bounds__(64) void k_cand_export(Ctx c, int ch0, int ch1) {
    const int lb = work_block();
    const int ch = ch0 + lb / c.nbands, bd = lb % c.nbands;
    if (ch >= ch1) return;
    const int lane = (int)threadIdx.x;
    const int cs = ch * c.C2, ce = min(cs + c.C2, c.n);
    const int H = c.H, OFF = c.X0 * H;
    const int64_t bi = (int64_t)ch * (c.nbands + 1) + bd;
    const int w0 = c.bstart[bi], w1 = c.bstart[bi + 1];
    int cnt = 0;  // (wave-uniform)
    for (int wb = w0; wb < w1; wb += 64) {
        const int w = wb + lane;
        bool keep = false;
        int4 rec = make_int4(0, 0, 0, 0);
        if (w < w1) {
            const int4 fd = c.fdesc[w];  // {event, x, y, t}
            const int nx = c.link[fd.x].z;
            if (nx >= ce && c.evf[fd.x].L > 0) {
                keep = true;
                rec = make_int4(fd.x, fd.y * H + fd.z - OFF, fd.w, nx);
            }
        }
        const uint64_t bal = __ballot(keep);
        if (keep) c.s2x[w0 + mbcnt64(bal, cnt)] = rec;
        cnt += (int)__popcll(bal);
    }
    if (lane == 0) c.s2b[bi] = cnt;
}

// One wavefront (= one workgroup: it slots in as the pooling waves free theirs)
// per (pooling chunk, band of columns) of chunks [ch0, ch1).  A band's cells
// [b * bandc * H, ...) start on a candidate-group boundary (bandc * H is a
// multiple of 256), so its bitmap words and their group-local offsets are its
// own; its events of any chunk are one range of the work order (bstart).
__global__ __launch_bounds__(64) void k_cand(Ctx c, int ch0, int ch1) {
    extern __shared__ uint64_t s_bm[];  // the band's bitmap words
    const int lb = work_block();  // XCD-contiguous: neighbouring bands share an L2
    const int ch = ch0 + lb / c.nbands, bd = lb % c.nbands;
    if (ch >= ch1) return;
    const int lane = (int)threadIdx.x;
    const int H = c.H;
    const uint32_t qa = (uint32_t)bd * (uint32_t)c.bandc * (uint32_t)H;
    const uint32_t qb = (uint32_t)min((int64_t)qa + (int64_t)c.bandc * H, c.WH);
    const int nw = (int)((qb - qa + 63) >> 6);
    for (int i = lane; i < nw; i += 64) s_bm[i] = 0;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const int n = c.n, C2 = c.C2;
    const int cs = ch * C2, ce = min(cs + C2, n);
    const int64_t lo = (int64_t)c.ctmin[ch] - (int64_t)kKillUs, hi = (int64_t)c.ctmax[ch] + (int64_t)kKillUs;
    const int cap = (int)(qb - qa);
    int32_t *scr = c.cscr + (int64_t)(ch - ch0) * c.WH + qa;  // this band's item slots in the chunk's scratch
    const int OFF = c.X0 * H;
    int cnt = 0;  // (wave-uniform)
    auto push = [&](bool keep, uint32_t q, int item) {
        const uint64_t bal = __ballot(keep);
        if (keep) {
            atomicOr((unsigned long long *)&s_bm[(q - qa) >> 6], 1ull << (q & 63));
            const int i = mbcnt64(bal, cnt);
            if (i < cap) scr[i] = item;  // (a cell is an item at most once: i < cap always)
        }
        cnt += (int)__popcll(bal);
    };
    const int32_t *bsr = c.bstart + (int64_t)bd;
    const int64_t bstride = c.nbands + 1;
    // S1: first events of the chunk at their cells
    {
        const int w0 = bsr[ch * bstride], w1 = bsr[ch * bstride + 1];
        for (int wb = w0; wb < w1; wb += 64) {
            const int w = wb + lane;
            bool keep = false;
            uint32_t q = 0;
            int e = 0;
            if (w < w1) {
                const int4 fd = c.fdesc[w];  // {event, x, y, t}
                e = fd.x;
                q = (uint32_t)(fd.y * H + fd.z - OFF);
                const int4 lk = c.link[e];
                if (lk.y < cs) {
                    if (lk.z < ce) keep = true;
                    else {
                        const FlowCell *sp = lk.y >= 0 ? &c.evf[lk.y] : &c.fsnap[q];
                        const double Le = c.evf[e].L, Ls = sp->L;
                        const int64_t ts = (int64_t)sp->t;
                        keep = Le > 0 || (Ls > 0 && ts > lo && ts < hi);
                    }
                }
            }
            push(keep, q, e);
        }
    }
    // S2: the last events before the chunk at untouched cells, from the chunks
    // whose stamps reach the kill window: their exported sources (the events
    // last at their cell in their own chunk with a valid flow, k_cand_export),
    // 16 B each, in work order -- a superset of this chunk's S2 from them
    for (int cp = c.cbk[ch]; cp < ch; ++cp) {
        if (!((int64_t)c.ctmax[cp] > lo && (int64_t)c.ctmin[cp] < hi)) continue;
        const int x0 = bsr[cp * bstride], x1 = x0 + c.s2b[cp * bstride + bd];
        for (int xb = x0; xb < x1; xb += 64) {
            const int x = xb + lane;
            bool keep = false;
            uint32_t q = 0;
            int e = 0;
            if (x < x1) {
                const int4 r = c.s2x[x];  // {event, cell, stamp, next event at the cell}
                const int64_t te = (int64_t)(uint32_t)r.z;
                e = r.x;
                q = (uint32_t)r.y;
                keep = te > lo && te < hi && r.w >= ce;
            }
            push(keep, q, e);
        }
    }
    // S3: call-start snapshots of cells the call has not touched before ce
    {
        const int ns = c.cinfo[kCiCount];
        if (ns > 0 && (int64_t)(uint32_t)c.cinfo[kCiLMax] > lo && (int64_t)(uint32_t)c.cinfo[kCiLMin] < hi) {
            for (int i0 = 0; i0 < ns; i0 += 64) {
                const int i = i0 + lane;
                bool keep = false;
                uint32_t q = 0;
                if (i < ns) {
                    const int4 en = c.slist[i];
                    q = (uint32_t)en.x;
                    const int64_t ft = (int64_t)(uint32_t)en.y;
                    keep = q >= qa && q < qb && ft > lo && ft < hi && en.z >= ce;
                }
                push(keep, q, ~(int)q);
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // bitmap words with the slot of their first candidate: the band's
    // candidates take slots [qa, qa + count) in cell order (band-contiguous, so
    // that a pooling row inside the band is one slot range: Ctx::band_slots)
    const int buf = (c.ring0 + ch) % c.NB;
    BmWord *bw = c.bw_ring + (int64_t)buf * c.nwords;
    const int64_t wbase = (int64_t)qa >> 6;
    uint32_t *s_wo = reinterpret_cast<uint32_t *>(s_bm + nw);
    {
        uint32_t carry = qa;  // (wave-uniform)
        for (int i0 = 0; i0 < nw; i0 += 64) {
            const int i = i0 + lane;
            const uint64_t m = i < nw ? s_bm[i] : 0ull;
            const int v = (int)__popcll(m);
            const int incl = wave_incl_scan(v);
            const uint32_t wo = carry + (uint32_t)(incl - v);
            if (i < nw) {
                s_wo[i] = wo;
                BmWord bv;
                bv.bm = m;
                bv.wo = wo;
                bv.pad = 0;
                bw[wbase + i] = bv;
            }
            carry += (uint32_t)__builtin_amdgcn_readlane(incl, 63);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // the records
    cnt = min(cnt, cap);
    CandHdr *hr = c.hdr_ring + (int64_t)buf * c.cstride;
    CandVal *vr = c.val_ring + (int64_t)buf * c.cstride;
    for (int i = lane; i < cnt; i += 64) {
        const int item = scr[i];
        CandHdr hd;
        CandVal v;
        uint32_t q;
        if (item >= cs) {  // S1
            const int e = item;
            q = c.pix[e];
            const int4 lk = c.link[e];
            const FlowCell fe = c.evf[e];
            const FlowCell sn = lk.y >= 0 ? c.evf[lk.y] : c.fsnap[q];
            hd.lin = q | (sn.L > 0 ? kCandSnapOk : 0u) | (fe.L > 0 ? kCandOneOk : 0u);
            hd.e1 = e;
            hd.t_snap = sn.t;
            hd.t1 = fe.t;
            v.L_snap = sn.L; v.Lc_snap = sn.Lc; v.Ls_snap = sn.Ls;
            v.L1 = fe.L; v.Lc1 = fe.Lc; v.Ls1 = fe.Ls;
            v.run_lo = lk.x;
            v.run_hi = lk.x;
            if (lk.z < ce) {  // more than one event at the cell in the chunk
                hd.lin |= kCandMore;
                const int e2 = lk.z;
                const int4 lk2 = c.link[e2];
                if (lk2.z < ce) {  // more than two: the run's last in-chunk position in P
                    hd.lin |= kCandMore2;
                    int a = lk2.x + 1, b = c.pend[q];  // P[a] = the third event < ce; ids ascend along the run
                    while (a < b) {
                        const int m = (a + b + 1) >> 1;
                        if (c.P[m] < ce) a = m;
                        else b = m - 1;
                    }
                    v.run_hi = a;
                } else {  // exactly two: the second inline
                    const FlowCell f2 = c.evf[e2];
                    v.run_lo = (int32_t)((uint32_t)e2 | (f2.L > 0 ? 0x80000000u : 0u));
                    v.run_hi = (int32_t)f2.t;
                }
            }
        } else {  // S2 (an earlier event) or S3 (a call-start snapshot): untouched in the chunk
            q = item >= 0 ? c.pix[item] : (uint32_t)~item;
            const FlowCell sn = item >= 0 ? c.evf[item] : c.fsnap[q];
            hd.lin = q | kCandSnapOk;
            hd.e1 = INT_MAX;
            hd.t_snap = sn.t;
            hd.t1 = 0;
            v.L_snap = sn.L; v.Lc_snap = sn.Lc; v.Ls_snap = sn.Ls;
            v.L1 = 0.0; v.Lc1 = 0.0; v.Ls1 = 0.0;
            v.run_lo = 0;
            v.run_hi = 0;
        }
        const int wi = (int)((q - qa) >> 6);
        const uint32_t slot = s_wo[wi] + (uint32_t)__popcll(s_bm[wi] & ((1ull << (q & 63)) - 1));
        hr[slot] = hd;
        if (item >= cs) {
            vr[slot] = v;
        } else {  // untouched in the chunk (e1 = INT_MAX): the pooling reads the snapshot only
            vr[slot].L_snap = v.L_snap;
            vr[slot].Lc_snap = v.Lc_snap;
            vr[slot].Ls_snap = v.Ls_snap;
        }
    }
}

// After a call's last k_cand: every cell's flow snapshot becomes its last
// event's flow, P[pend[q]] (k_chain advances them itself).  One thread per
// cell: 4 B per cell plus two gathers per touched cell, where a pass over the
// events' links read 16 B per event (0.96 GB per 50M-event call, PMC).
__global__ void k_cand_commit(Ctx c) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= c.WH) return;
    const int k = c.pend[q];
    if (k < 0) return;
    FlowCell f = c.evf[c.P[k]];
    f.pad = 0;
    c.fsnap[q] = f;
    c.ftime[q] = f.L > 0 ? (int64_t)f.t : -1;
}

// Last event with id <= e over a candidate's in-chunk run P[lo..hi] (P[lo] <= e).
__device__ __forceinline__ int run_search_bounds(const Ctx &c, int lo, int hi, int e) {
    if (c.P[hi] <= e) return hi;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (c.P[mid] <= e) lo = mid;
        else hi = mid;
    }
    return lo;
}

// Element i of an array whose byte offsets fit 32 bits, addressed as a
// wave-uniform base plus a zero-extended 32-bit offset (the global_load saddr
// form: one VGPR of offset instead of a sign-extended 64-bit address per lane).
template <class T>
__device__ __forceinline__ const T &at32(const T *base, uint32_t i) {
    return *reinterpret_cast<const T *>(reinterpret_cast<const char *>(base) + (uint32_t)(i * (uint32_t)sizeof(T)));
}

// Max over the 64 lanes (exact).
__device__ __forceinline__ double wave_max(double v) {
    v = fmax(v, xch<0>(v));
    v = fmax(v, xch<1>(v));
    v = fmax(v, xch<2>(v));
    v = fmax(v, xch<3>(v));
    v = fmax(v, xch<4>(v));
    v = fmax(v, xch<5>(v));
    return v;
}

// Multiscale pooling (computeTrueFlow, vFlow.cpp:952-1210): one wavefront per
// valid event.
//   Window: rows i in [x-M, x+M] span x-major cell ranges [i*H + j_lo, i*H + j_hi]
//   with j clipped to W-1 as the reference does (vFlow.cpp:1000/1113): for W > H
//   a row runs into the next column (aliasing kept); indices >= W*H do not
//   contribute.  Each row is a contiguous slice of the chunk's candidate list
//   (bitmap popcount prefix); the slices are flattened (pool_rows).
//   Then one pass over the flattened candidates, 64 per step, in raster order:
//   resolve each cell's state as of e, load the values of the contributors
//   (valid flow, |dt| < 500 us), stage them in LDS in rank order (ballot) and
//   fold them into the per-scale sums in the reference's order (pool_one).
// The summation order depends only on the contributor list, so results are
// bitwise independent of chunking and streaming splits.
// Fold of 8 staged entries into this lane's sum: entry u (smallest scale k0 =
// byte u of kw0:kw1) is added iff kk >= k0, as an exec-masked v_add_f64: the
// member test runs once per entry for all lanes (v_cmp into an SGPR mask, all
// 8 before any exec change), then each add executes on the member lanes only,
// bitwise the conditional add of the reference (vFlow.cpp:1005-1008) and one
// fp64 add per entry on the dependency chain (the masked-fma form costs a
// compare, a select and an fma).  exec is restored before the asm ends.  The
// masks are subsets of exec (v_cmp writes 0 for inactive lanes), so exec is set
// with s_mov_b64, which leaves SCC alone: the surrounding code may hold a
// loop condition there (s_and_b64 would clobber it).  (The same sum as a
// masked fma, fma(v, m, acc) with m in {0, 1}, is bitwise equal -- acc starts
// at +0 and a round-to-nearest sum is -0 only when both addends are -- but
// costs a compare, a select and an fma per entry.)
// The scalar-mask folds below set exec to masks computed from scratch, valid
// only under a full exec at entry; -DFARMS_CHECK_EXEC traps on any other.
__device__ __forceinline__ void fold_exec_check() {
#ifdef FARMS_CHECK_EXEC
    if (__builtin_amdgcn_read_exec() != ~0ull) __builtin_trap();
#endif
}
__device__ __forceinline__ void fold8(double &acc, int kk, uint32_t kw0, uint32_t kw1, const double (&v)[8]) {
    uint64_t m0, m1, m2, m3, m4, m5, m6, m7, sv;
    asm volatile(
        "v_cmp_ge_i32_sdwa %[m0], %[kk], %[kw0] src0_sel:DWORD src1_sel:BYTE_0\n"
        "v_cmp_ge_i32_sdwa %[m1], %[kk], %[kw0] src0_sel:DWORD src1_sel:BYTE_1\n"
        "v_cmp_ge_i32_sdwa %[m2], %[kk], %[kw0] src0_sel:DWORD src1_sel:BYTE_2\n"
        "v_cmp_ge_i32_sdwa %[m3], %[kk], %[kw0] src0_sel:DWORD src1_sel:BYTE_3\n"
        "v_cmp_ge_i32_sdwa %[m4], %[kk], %[kw1] src0_sel:DWORD src1_sel:BYTE_0\n"
        "v_cmp_ge_i32_sdwa %[m5], %[kk], %[kw1] src0_sel:DWORD src1_sel:BYTE_1\n"
        "v_cmp_ge_i32_sdwa %[m6], %[kk], %[kw1] src0_sel:DWORD src1_sel:BYTE_2\n"
        "v_cmp_ge_i32_sdwa %[m7], %[kk], %[kw1] src0_sel:DWORD src1_sel:BYTE_3\n"
        "s_mov_b64 %[sv], exec\n"
        "s_mov_b64 exec, %[m0]\n"
        "v_add_f64 %[acc], %[acc], %[v0]\n"
        "s_mov_b64 exec, %[m1]\n"
        "v_add_f64 %[acc], %[acc], %[v1]\n"
        "s_mov_b64 exec, %[m2]\n"
        "v_add_f64 %[acc], %[acc], %[v2]\n"
        "s_mov_b64 exec, %[m3]\n"
        "v_add_f64 %[acc], %[acc], %[v3]\n"
        "s_mov_b64 exec, %[m4]\n"
        "v_add_f64 %[acc], %[acc], %[v4]\n"
        "s_mov_b64 exec, %[m5]\n"
        "v_add_f64 %[acc], %[acc], %[v5]\n"
        "s_mov_b64 exec, %[m6]\n"
        "v_add_f64 %[acc], %[acc], %[v6]\n"
        "s_mov_b64 exec, %[m7]\n"
        "v_add_f64 %[acc], %[acc], %[v7]\n"
        "s_mov_b64 exec, %[sv]\n"
        : [acc] "+v"(acc), [m0] "=&s"(m0), [m1] "=&s"(m1), [m2] "=&s"(m2), [m3] "=&s"(m3), [m4] "=&s"(m4),
          [m5] "=&s"(m5), [m6] "=&s"(m6), [m7] "=&s"(m7), [sv] "=&s"(sv)
        : [kk] "v"(kk), [kw0] "v"(kw0), [kw1] "v"(kw1), [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]),
          [v3] "v"(v[3]), [v4] "v"(v[4]), [v5] "v"(v[5]), [v6] "v"(v[6]), [v7] "v"(v[7]));
}
// The same fold with the member masks from the scalar unit (kSaluFold): the
// entries' shift amounts 4 k0 are bytes of sw0:sw1 (SGPRs), entry u's members
// are the lanes >= 4 k0, so exec = -1 << 4 k0 is one s_lshl_b64 (it reads bits
// [5:0] of its shift operand: byte u is reached by a right shift of 8 (u % 4)).
// The fold's only VALU instructions are then the exec-masked v_add_f64s (the
// v_cmp per entry was about 157 of k_pool's ~1,115 VALU instructions per valid
// event at C3, round 4).  Bitwise the fold8 sums: the same adds on the same
// lanes.  The shifted masks are NOT intersected with the exec at entry: every
// caller runs with a full exec (wave-uniform control flow), which
// fold_exec_check asserts in a -DFARMS_CHECK_EXEC build.  (Intersecting them,
// one s_and_b64 before each add, measured C3 69.2 against 66.7 ms: the exec
// write sits on the add chain.)  The shifts write SCC, hence the clobber.
__device__ __forceinline__ void fold8_salu(double &acc, uint32_t sw0, uint32_t sw1, const double (&v)[8]) {
    fold_exec_check();
    uint64_t sv;
    uint32_t t;
    asm volatile(
        "s_mov_b64 %[sv], exec\n"
        "s_lshl_b64 exec, -1, %[w0]\n"
        "v_add_f64 %[acc], %[acc], %[v0]\n"
        "s_lshr_b32 %[t], %[w0], 8\n"
        "s_lshl_b64 exec, -1, %[t]\n"
        "v_add_f64 %[acc], %[acc], %[v1]\n"
        "s_lshr_b32 %[t], %[w0], 16\n"
        "s_lshl_b64 exec, -1, %[t]\n"
        "v_add_f64 %[acc], %[acc], %[v2]\n"
        "s_lshr_b32 %[t], %[w0], 24\n"
        "s_lshl_b64 exec, -1, %[t]\n"
        "v_add_f64 %[acc], %[acc], %[v3]\n"
        "s_lshl_b64 exec, -1, %[w1]\n"
        "v_add_f64 %[acc], %[acc], %[v4]\n"
        "s_lshr_b32 %[t], %[w1], 8\n"
        "s_lshl_b64 exec, -1, %[t]\n"
        "v_add_f64 %[acc], %[acc], %[v5]\n"
        "s_lshr_b32 %[t], %[w1], 16\n"
        "s_lshl_b64 exec, -1, %[t]\n"
        "v_add_f64 %[acc], %[acc], %[v6]\n"
        "s_lshr_b32 %[t], %[w1], 24\n"
        "s_lshl_b64 exec, -1, %[t]\n"
        "v_add_f64 %[acc], %[acc], %[v7]\n"
        "s_mov_b64 exec, %[sv]\n"
        : [acc] "+v"(acc), [sv] "=&s"(sv), [t] "=&s"(t)
        : [w0] "s"(sw0), [w1] "s"(sw1), [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]),
          [v4] "v"(v[4]), [v5] "v"(v[5]), [v6] "v"(v[6]), [v7] "v"(v[7])
        : "scc");
}
// Fold of 8 staged entries whose packed k0 bytes (kenc: 4 k0 for the scalar
// masks) are kw0:kw1, into this lane's sum (lane layout: kSaluFold).
template <int K>
__device__ __forceinline__ void fold8_k(double &acc, int kk, uint32_t kw0, uint32_t kw1, const double (&v)[8]) {
    if constexpr (kSaluFold<K>)
        fold8_salu(acc, __builtin_amdgcn_readfirstlane(kw0), __builtin_amdgcn_readfirstlane(kw1), v);
    else
        fold8(acc, kk, kw0, kw1, v);
}
// Row setup of a pooling window: the flattened candidate slices of rows
// [i_lo, i_lo + nrows) (nrows <= 128), cells j in [j_lo, j_hi] of each row
// (x-major; j already clipped to W-1 as vFlow.cpp:1000/1113 do, so for W > H a
// row runs into the next column; indices >= W*H do not contribute).  Writes
// s_start (bit f set iff a non-empty row segment starts at flattened position
// f), s_row (the non-empty segments in order: {row, candidate index - flattened
// index}).  Returns the flattened length.  LDS private to the calling wave.
// The slot layouts of a chunk's candidate buffer (pool_rows / pool_rows2 MODE).
constexpr int kSlotsGroup = 0, kSlotsBand = 1, kSlotsBandFlat = 2;
// kSlotsBand: the local cell where the band after the one holding a window
// row's first cell starts, for the row of absolute x-row i (its first cell is
// in local x-row i - X0, or in local cell 0 when the row starts left of the
// stored region).  A row range is at most 2M + 1 <= 127 cells and a band at
// least 256 (bandc H, whole candidate groups), so a range splits at most once,
// and there.  The W - 1 clip can carry a range over more than one x-row (H <=
// M): the band start is then not always the next x-row's first cell.
__device__ __forceinline__ int band_split(const Ctx &c, int i) {
    const int cs = i - c.X0;
    return (((cs < 0 ? 0 : cs) | (c.bandc - 1)) + 1) * c.H;
}
template <int MODE>  // (the slot layout: see pool_rows2)
__device__ __forceinline__ int pool_rows(const Ctx &c, int buf, int lane, int i_lo, int nrows, int j_lo, int j_hi,
                                         uint64_t *s_start, uint32_t *s_row) {
    const int H = c.H;
    const int WHl = (int)c.WH, OFF = c.X0 * c.H;  // local cell = global cell - OFF
    const int WHs = (int)c.WHs;
    // ---- per-row candidate slices: flattened start of each non-empty row as a
    // bit of s_start, and its candidate offset in s_row
    uint32_t *const sbits = reinterpret_cast<uint32_t *>(s_start);
    {
        const int nw = ((nrows * (j_hi - j_lo + 1) + 63) >> 6) + 1;  // bound on the flattened length, in words (+1)
        for (int i = lane; i < nw; i += 64) s_start[i] = 0;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // A row's cell range maps to one candidate slice per candidate group it
    // overlaps (ranges are shorter than a group: at most two segments; the
    // second starts at its group's first slot, whose index is the group's
    // first cell index).  Lane l handles rows l and l + 64 (2M+1 <= 127): the
    // lookups of both are in flight before either is used.
    // All six lookups of both rows are unconditional loads from clamped word
    // indices (a load under a branch would be waited for at the branch end).
    int a0[2], n0[2], a1[2], n1[2];
    const BmWord *bwb = c.bw_ring + (int64_t)buf * c.nwords;
    const int wmax = (int)c.nwords - 1;
    int lo_[2], hi0_[2], hi1_[2], gb_[2];
    bool has_[2], str_[2];
    uint64_t bA[2], bB[2], bC[2];
    uint32_t oA[2], oB[2], oC[2];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
        const int r = lane + 64 * hh;
        const int base = (i_lo + (r < nrows ? r : 0)) * H;
        int l1 = base + j_hi;
        if (l1 > WHs - 1) l1 = WHs - 1;  // past the end of the sensor: no contribution
        int l0 = base + j_lo - OFF;
        l1 -= OFF;
        if (l0 < 0) l0 = 0;               // outside the stored region: never visited
        if (l1 > WHl - 1) l1 = WHl - 1;
        has_[hh] = r < nrows && l0 <= l1;
        int gb;
        if constexpr (MODE == kSlotsGroup) {
            gb = l1 & ~(kGroupCells - 1);            // first cell of l1's group
            str_[hh] = has_[hh] && l0 < gb;          // the range crosses into l1's group
        } else if constexpr (MODE == kSlotsBand) {
            gb = band_split(c, i_lo + r);            // the first band start past l0
            str_[hh] = has_[hh] && gb <= l1;
        } else {
            gb = 0;
            str_[hh] = false;
        }
        lo_[hh] = l0; gb_[hh] = gb;
        hi0_[hh] = str_[hh] ? gb - 1 : l1;       // end of the first segment
        hi1_[hh] = l1;
        // word indices clamped for the loads only (a row without cells keeps has_
        // false): l0 >= 0 here, and a negative l1 wraps to wmax as unsigned
        const uint32_t wa = min((uint32_t)l0 >> 6, (uint32_t)wmax), wc = min((uint32_t)l1 >> 6, (uint32_t)wmax);
        const BmWord A = at32(bwb, wa), C = at32(bwb, wc);
        bA[hh] = A.bm; oA[hh] = A.wo;
        bC[hh] = C.bm; oC[hh] = C.wo;
        if constexpr (MODE != kSlotsBandFlat) {
            const uint32_t wb = min((uint32_t)hi0_[hh] >> 6, (uint32_t)wmax);
            const BmWord B = at32(bwb, wb);
            bB[hh] = B.bm; oB[hh] = B.wo;
        } else {
            bB[hh] = 0; oB[hh] = 0;
        }
    }
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
        // candidate index of the first candidate >= L (lo) / one past the last <= L (hi)
        const int lo = (int)(oA[hh] + (uint32_t)__popcll(bA[hh] & ((1ull << (lo_[hh] & 63)) - 1)));
        const int h1 = (int)(oC[hh] + (uint32_t)__popcll(bC[hh] & ((2ull << (hi1_[hh] & 63)) - 1)));
        a0[hh] = lo;
        a1[hh] = gb_[hh];
        if constexpr (MODE == kSlotsBandFlat) {
            n0[hh] = has_[hh] ? h1 - lo : 0;
            n1[hh] = 0;
        } else {
            const int h0 = (int)(oB[hh] + (uint32_t)__popcll(bB[hh] & ((2ull << (hi0_[hh] & 63)) - 1)));
            n0[hh] = has_[hh] ? h0 - lo : 0;
            n1[hh] = str_[hh] ? h1 - gb_[hh] : 0;
        }
    }
    int carry = 0, nz = 0;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
        if (64 * hh >= nrows) break;
        const int r = lane + 64 * hh;
        const int cnt = n0[hh] + n1[hh];
        const int incl = wave_incl_scan(cnt);
        const int start = carry + incl - cnt;
        const uint64_t b0 = __ballot(n0[hh] > 0), b1 = MODE == kSlotsBandFlat ? 0ull : __ballot(n1[hh] > 0);
        int idx = MODE == kSlotsBandFlat ? mbcnt64(b0, nz) : mbcnt64(b1, mbcnt64(b0, nz));
        if (n0[hh] > 0) {
            s_row[idx++] = ((uint32_t)r << 25) | (uint32_t)(a0[hh] - start + kRowBias);
            atomicOr(&sbits[start >> 5], 1u << (start & 31));
        }
        if (n1[hh] > 0) {
            const int st1 = start + n0[hh];
            s_row[idx] = ((uint32_t)r << 25) | (uint32_t)(a1[hh] - st1 + kRowBias);
            atomicOr(&sbits[st1 >> 5], 1u << (st1 & 31));
        }
        nz += (int)__popcll(b0) + (int)__popcll(b1);
        carry += __builtin_amdgcn_readlane(incl, 63);
    }
    // the LDS arrays are private to this wave: a wavefront-scope fence orders
    // the writes above before the reads below
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    return carry;
}

// Pooling of one valid owned event e at (ex, ey, teu) by the calling wave from
// the row table built by pool_rows (rows from absolute row row_i0): flattened
// candidates [0, total).  One pass, 64 candidates per step, software-pipelined:
//   step s resolves the headers of s (loaded during step s-1: the cell's state
//   as of e -- snapshot, first in-chunk flow, or a run search when the cell
//   fired more than once in the chunk), keeps the contributors (valid flow,
//   |t_e - t_cell| < 500 us, vFlow.cpp:1002/1115) and issues the loads of
//   their values {L, L cos, L sin} and of the headers of s+1; meanwhile the
//   contributors of s-1 (values landed) go to LDS in rank order and are folded.
//   Fold: lane g*K + kk adds entry after entry to its sum of quantity g (L,
//   L cos, L sin) of scale kk, members only (k0 <= kk): vFlow.cpp:998-1021
//   accumulates each scale from 0, cell by cell, i ascending then j ascending,
//   and the staged entries are exactly the contributors of the largest window
//   in that order (row slices in row order, ascending cells within a row; a
//   cell the W-1 clip aliases into two rows appears twice, as the reference
//   visits it twice).  So every per-scale sum, mean and the first strict
//   maximum are bitwise the reference's given the same local flows.  Lanes
//   3K + kk fold 1.0 per member: the contributor count of scale kk, exact.
// LDS (private to the wave): s_val / s_k0 the values {L, L cos, L sin, 1} and k0 of one step's
// 64 staged entries (contributors first, in rank order).
template <int K>
__device__ __forceinline__ void pool_finish(const Ctx &c, int e, int lane, double acc, int scanned, int ncon_total);
#ifdef FARMS_POOL_STAMPS
#define POOL_ST_PARAM , PoolSt &pool_st
#define POOL_ST_ARG , pool_st
#else
#define POOL_ST_PARAM
#define POOL_ST_ARG
#endif
template <int K>
__device__ __forceinline__ void pool_one(const Ctx &c, int e, int ex, int ey, uint32_t teu, int buf, int lane,
                                         int row_i0, int total, int ev0, const uint64_t *s_start,
                                         const uint32_t *s_row, double *s_val, uint8_t *s_k0 POOL_ST_PARAM) {
    static_assert(4 * K <= 64, "one lane per (quantity, scale)");
    const CandHdr *chdr = c.hdr_ring + (int64_t)buf * c.cstride;
    const CandVal *cval = c.val_ring + (int64_t)buf * c.cstride;
    const int H = c.H, J = c.J;
    const int OFF = c.X0 * c.H;
    // serial mode: the own cell is pooled with the stamp its lastEventTime still
    // holds (the previous event's), not the event's own (vFlow.cpp:790 vs :264)
    const uint32_t own_lin = c.serial ? (uint32_t)((ex - c.X0) * H + ey) : 0xFFFFFFFFu;
    const uint32_t own_tprev = c.serial ? (uint32_t)c.link[e].w : 0u;
    (void)ev0;
    // quantity g of scale kk, g = 0..3 (L, L cos, L sin, and the contributor
    // count as a sum of 1.0: exact), on lane 4 kk + g (kSaluFold) or g K + kk;
    // lanes past 4K fold junk.  s_k0 holds kenc(k0): 4 k0 for the scalar masks.
    constexpr bool SF = kSaluFold<K>;
    const int grp = SF ? (lane & 3) : (lane / K < 3 ? lane / K : 3);
    const int kk = SF ? (lane >> 2) : lane - grp * K;
    constexpr int kenc_mul = SF ? 4 : 1;
    constexpr int NH = kPoolHalves;  // candidates per lane per step: a step covers 64 * NH positions
#pragma unroll
    for (int i = lane; i < kPoolSlots; i += 64) s_val[4 * i + 3] = 1.0;  // the count's "value" (staging never overwrites it)
    double acc = 0.0;
    int ncon_total = 0;
    // lanes without a contributor load the event's own flow (a valid address,
    // finite values that a non-member fold adds as +0)
    const double *const vdummy = reinterpret_cast<const double *>(c.evf + e);
    // Flattened position f = f0 + 64 h + lane: its segment is the last non-empty
    // one starting at or before f, i.e. the (number of segment starts <= f)-th.
    int mbase = 0;
    auto locate = [&](int f0, int (&row)[NH], int (&k)[NH]) {
#pragma unroll
        for (int h = 0; h < NH; ++h) {
            const uint64_t mk = s_start[(f0 >> 6) + h];
            const int m = mbase + (int)__popcll(mk & ((2ull << lane) - 1)) - 1;
            mbase += (int)__popcll(mk);
            const uint32_t rs = s_row[m < 0 ? 0 : m];
            row[h] = (int)(rs >> 25);
            k[h] = f0 + 64 * h + lane + (int)(rs & 0x1FFFFFFu) - kRowBias;
        }
    };
    int rc[NH], kc[NH];
    CandHdr hc[NH];
#pragma unroll
    for (int h = 0; h < NH; ++h) { rc[h] = 0; kc[h] = 0; hc[h] = CandHdr{}; }
    if (total > 0) {
        locate(0, rc, kc);
#pragma unroll
        // (lanes past the end load lane 0's header: no exec mask, and no
        // second line -- a fixed index would send every wave to one L2 channel)
        for (int h = 0; h < NH; ++h)
            hc[h] = at32(chdr, 64 * h + lane < total ? (uint32_t)kc[h] : (uint32_t)__builtin_amdgcn_readfirstlane(kc[0]));
    }
    // the previous step's contributors: ballots, values, smallest scales
    uint64_t pbal[NH];
    double pv[NH][3];
    int pk0[NH];
#pragma unroll
    for (int h = 0; h < NH; ++h) { pbal[h] = 0; pv[h][0] = pv[h][1] = pv[h][2] = 0.0; pk0[h] = K; }
    int staged = 0;  // (wave-uniform) staged entries not yet folded, at slots [0, staged)
#ifdef FARMS_POOL_STAMPS
    uint64_t st_fold = 0, st_steps = 0, st_groups = 0;
#endif
    for (int f0 = 0;; f0 += 64 * NH) {
        const bool have = f0 < total;  // wave-uniform
        bool con[NH];
        int k0[NH];
        const double *vp[NH];
#pragma unroll
        for (int h = 0; h < NH; ++h) {
            con[h] = false;
            k0[h] = K;
            vp[h] = vdummy;
            if (have && f0 + 64 * h + lane < total) {
                const CandHdr &hd = hc[h];
                uint32_t tq;
                bool ok;
                if (hd.e1 > e) { ok = (hd.lin & kCandSnapOk) != 0; tq = hd.t_snap; vp[h] = &cval[kc[h]].L_snap; }
                else if (!(hd.lin & kCandMore)) { ok = (hd.lin & kCandOneOk) != 0; tq = hd.t1; vp[h] = &cval[kc[h]].L1; }
                else if (!(hd.lin & kCandMore2)) {  // two events at the cell inside the chunk: the second inline
                    const int2 r2 = *reinterpret_cast<const int2 *>(&cval[kc[h]].run_lo);
                    const int e2 = r2.x & 0x7FFFFFFF;
                    if (e2 > e) { ok = (hd.lin & kCandOneOk) != 0; tq = hd.t1; vp[h] = &cval[kc[h]].L1; }
                    else { ok = r2.x < 0; tq = (uint32_t)r2.y; vp[h] = &c.evf[e2].L; }
                }
                else {  // more events at the cell inside the chunk: search its run
                    const CandVal &cv = cval[kc[h]];
                    const int sev = c.P[run_search_bounds(c, cv.run_lo, cv.run_hi, e)];
                    const FlowCell fe = c.evf[sev];
                    ok = fe.L > 0; tq = fe.t; vp[h] = &c.evf[sev].L;
                }
                if ((hd.lin & kCandLinMask) == own_lin) tq = own_tprev;
                // |t_e - t_cell| < 500 us (vFlow.cpp:1002/1115), exact on integers
                const int64_t dt = (int64_t)teu - (int64_t)tq;
                const int i = row_i0 + rc[h];
                // (i * H < 2^24: the full-rate 24-bit multiply)
                const int j = (int)(hd.lin & kCandLinMask) + OFF - (int)__umul24((uint32_t)i, (uint32_t)H);
                if (ok && (uint64_t)(dt + 499) < 999u) {
                    const int di = i > ex ? i - ex : ex - i, dj = j > ey ? j - ey : ey - j;
                    const int d = di > dj ? di : dj;
                    // smallest scale containing the cell, ceil(d / J), by a multiply-high with
                    // ceil(2^32 / J) (exact for d + J < 2^16; J = 1: d)
                    k0[h] = J == 1 ? d : (int)__umulhi((uint32_t)(d + J - 1), c.kmagic);
                    con[h] = true;
                }
            }
            if (!con[h]) vp[h] = vdummy;
        }
        // this step's values and the next step's headers: both in flight during
        // the fold below (unconditional loads: a load under a branch would be
        // waited for at the branch end)
        double v[NH][3];
#pragma unroll
        for (int h = 0; h < NH; ++h) { v[h][0] = vp[h][0]; v[h][1] = vp[h][1]; v[h][2] = vp[h][2]; }
        int rn[NH], kn[NH];
        CandHdr hn[NH];  // (past the last step: the current headers, never read)
#pragma unroll
        for (int h = 0; h < NH; ++h) { rn[h] = 0; kn[h] = 0; hn[h] = hc[h]; }
        if (f0 + 64 * NH < total) {  // (wave-uniform)
            locate(f0 + 64 * NH, rn, kn);
#pragma unroll
            for (int h = 0; h < NH; ++h)
                hn[h] = at32(chdr, f0 + 64 * (NH + h) + lane < total ? (uint32_t)kn[h]
                                                                      : (uint32_t)__builtin_amdgcn_readfirstlane(kn[0]));
        }
        // ---- stage and fold the previous step's contributors: they go to LDS
        // slots [staged, staged + cnt) in raster order (half 0 before half 1),
        // behind the entries the last step left unfolded; whole groups of 8
        // are folded and the rest (< 8) moves to slots [0, ...) for the next
        // step, so that only the event's last group is padded (every step's
        // last group was, before: ~8% of the fold's adds at C3)
        uint64_t pany = 0;
#pragma unroll
        for (int h = 0; h < NH; ++h) pany |= pbal[h];
        if (pany) {
            int cntb[NH], cnt = 0;
#pragma unroll
            for (int h = 0; h < NH; ++h) { cntb[h] = (int)__popcll(pbal[h]); cnt += cntb[h]; }
            // the previous fold's LDS reads are done (wave-private LDS)
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            int cbase = staged;
#pragma unroll
            for (int h = 0; h < NH; ++h) {
                if ((pbal[h] >> lane) & 1) {
                    const int slot = mbcnt64(pbal[h], cbase);
                    s_val[4 * slot] = pv[h][0]; s_val[4 * slot + 1] = pv[h][1]; s_val[4 * slot + 2] = pv[h][2];
                    s_k0[slot] = (uint8_t)(kenc_mul * pk0[h]);
                }
                cbase += cntb[h];
            }
            staged = cbase;
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            const int whole = staged & ~7;
            const uint32_t *k4p = reinterpret_cast<const uint32_t *>(s_k0);
#ifdef FARMS_POOL_STAMPS
            POOL_CLOCK(tf0);
            st_groups += whole >> 3;
            st_steps += 1;
#endif
            // (each group waits for its own LDS reads: reading group r + 8
            // while group r is added, in two register sets, measured slower,
            // C3 80.7 against 77.4 ms, profiles/r05_ab_fold_prefetch.log)
#pragma unroll 1
            for (int r = 0; r < whole; r += 8) {
                const uint32_t kw0 = k4p[r >> 2], kw1 = k4p[(r >> 2) + 1];
                double vv[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) vv[u] = s_val[4 * (r + u) + grp];
                fold8_k<K>(acc, kk, kw0, kw1, vv);
            }
#ifdef FARMS_POOL_STAMPS
            {
                POOL_CLOCK(tf1);
                st_fold += tf1 - tf0;
            }
#endif
            if (whole > 0 && staged > whole) {  // carry the rest to slots [0, staged - whole)
                const int rest = staged - whole;
                double m0 = 0.0, m1 = 0.0, m2 = 0.0;
                uint8_t mk = (uint8_t)K;
                if (lane < rest) {
                    m0 = s_val[4 * (whole + lane)]; m1 = s_val[4 * (whole + lane) + 1]; m2 = s_val[4 * (whole + lane) + 2];
                    mk = s_k0[whole + lane];
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                __builtin_amdgcn_wave_barrier();
                if (lane < rest) {
                    s_val[4 * lane] = m0; s_val[4 * lane + 1] = m1; s_val[4 * lane + 2] = m2;
                    s_k0[lane] = mk;
                }
            }
            staged -= whole;
            ncon_total += cnt;
        }
        if (!have) break;
#pragma unroll
        for (int h = 0; h < NH; ++h) {
            pbal[h] = __ballot(con[h]);
            pv[h][0] = v[h][0]; pv[h][1] = v[h][1]; pv[h][2] = v[h][2];
            pk0[h] = k0[h];
            hc[h] = hn[h]; rc[h] = rn[h]; kc[h] = kn[h];
        }
    }
    if (staged > 0) {  // the last group, padded with entries in no scale (k0 = K)
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (lane >= staged && lane < 8) s_k0[lane] = (uint8_t)(kenc_mul * K);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const uint32_t *k4p = reinterpret_cast<const uint32_t *>(s_k0);
        const uint32_t kw0 = k4p[0], kw1 = k4p[1];
        double vv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) vv[u] = s_val[4 * u + grp];
        fold8_k<K>(acc, kk, kw0, kw1, vv);
    }
#ifdef FARMS_POOL_STAMPS
    POOL_STAMP_ADD(3, st_fold);
    POOL_STAMP_ADD(6, st_steps);
    POOL_STAMP_ADD(7, st_groups);
    POOL_CLOCK(tp0);
#endif
    pool_finish<K>(c, e, lane, acc, total, ncon_total);
#ifdef FARMS_POOL_STAMPS
    POOL_CLOCK(tp1);
    POOL_STAMP_ADD(4, tp1 - tp0);
#endif
}

// Every per-scale sum of event e folded (lane g * K + kk holds quantity g of
// scale kk): the first strict max of the mean length over scales
// (vFlow.cpp:1023-1059) -- the winner is the lowest k whose mean equals the
// maximum, if it is > 0 -- and the event's global flow vector.
template <int K>
__device__ __forceinline__ void pool_finish(const Ctx &c, int e, int lane, double acc, int scanned, int ncon_total) {
    const int J = c.J;
    // the lane holding quantity g of scale k (pool_one's layout)
    auto at = [](int g, int k) { return kSaluFold<K> ? 4 * k + g : g * K + k; };
    const int kl = lane < K ? lane : 0;
    const double cnt_kk = __shfl(acc, at(3, kl), 64);  // contributors of scale lane
    const double len_kk = kSaluFold<K> ? __shfl(acc, at(0, kl), 64) : acc;
    const bool is_len = lane < K;
    const double mean = is_len && cnt_kk > 0 ? len_kk / cnt_kk : 0.0;
    const double maxv = wave_max(mean);
    const int mi = maxv > 0 ? __builtin_ctzll(__ballot(is_len && mean == maxv)) : 0;
    const double sx = __shfl(acc, at(1, mi), 64), sy = __shfl(acc, at(2, mi), 64), cnt_mi = __shfl(acc, at(3, mi), 64);
    // lane 0 takes Gx, lane 1 Gy: one division sequence for both
    if (lane < 2) {
        double g;
        if (maxv > 0) {
            g = (lane == 0 ? sx : sy) / cnt_mi;  // vFlow.cpp:1028-1029, 1067-1075
        } else {  // vFlow.cpp:1085-1094
            const FlowCell &self = c.evf[e];
            g = lane == 0 ? self.Lc : self.Ls;
        }
        (lane == 0 ? c.r_true : c.th_true)[e] = g;  // (RTrue, ThetaTrue) by k_true_polar, 64 events per wave
        if (lane == 0) {
            c.scale[e] = maxv > 0 ? mi * J : 0;
            if (c.dbg_tc) c.dbg_tc[e] = make_int2(scanned, ncon_total);
        }
    }
}

// Per-event pooling: the row table of the event's own window, then the event.
template <int K>
__device__ __forceinline__ void pool_event(const Ctx &c, int e, int ex, int ey, uint32_t teu, int buf, int lane,
                                           int ev0, uint64_t *s_start, uint32_t *s_row, double *s_val,
                                           uint8_t *s_k0 POOL_ST_PARAM) {
    const int W = c.W, M = c.M;
    const int i_lo = ex - M < 0 ? 0 : ex - M, i_hi = ex + M > W - 1 ? W - 1 : ex + M;
    const int j_lo = ey - M < 0 ? 0 : ey - M, j_hi = ey + M > W - 1 ? W - 1 : ey + M;
    POOL_CLOCK(tr0);
    int total;  // (the layout branch is wave-uniform: one event per wave)
    if (!c.band_slots) total = pool_rows<kSlotsGroup>(c, buf, lane, i_lo, i_hi - i_lo + 1, j_lo, j_hi, s_start, s_row);
    else if (j_hi >= c.H) total = pool_rows<kSlotsBand>(c, buf, lane, i_lo, i_hi - i_lo + 1, j_lo, j_hi, s_start, s_row);
    else total = pool_rows<kSlotsBandFlat>(c, buf, lane, i_lo, i_hi - i_lo + 1, j_lo, j_hi, s_start, s_row);
    POOL_CLOCK(tr1);
    POOL_STAMP_ADD(1, tr1 - tr0);
    pool_one<K>(c, e, ex, ey, teu, buf, lane, i_lo, total, ev0, s_start, s_row, s_val, s_k0 POOL_ST_ARG);
    POOL_CLOCK(tr2);
    POOL_STAMP_ADD(2, tr2 - tr1);
}

// One wavefront (= one workgroup, so that a finished event frees its slot at
// once) per work-order position of [c0, c1) (events of a chunk in tile order);
// invalid events and halo events (fitted here, pooled by their owner) leave at
// once.
#define FARMS_POOL_FLOOR_7 "v71"  // k_pool occupancy cap of 7 waves per SIMD (see k_pool)
#define FARMS_POOL_FLOOR_6 "v79"  // k_pool occupancy cap of 6 waves per SIMD
template <int K, bool W7>
__global__ __launch_bounds__(64) void k_pool(Ctx c, int c0, int c1) {
    // LDS per wave, sized for maxWindow M at launch: segment-start bitmap over
    // the flattened window, <= 2 row segments per window row, the values and
    // k0 of one step's 64 staged entries
    extern __shared__ __attribute__((aligned(16))) uint64_t s_dyn[];
    const int nbw = c.pool_bw, nrs = c.pool_rs;
    const int lane = threadIdx.x & 63;
    // Occupancy cap: the kernel allocates at least 72 VGPRs (W7: at most 7
    // pooling waves per SIMD) or 80 (6 waves).  The fit sweep's waves need the
    // room: each of its launches waits for its slowest wave, so crowding them
    // stretches the whole pipeline.  The optimum moves with the fit's weight: 6
    // waves/SIMD won while the fit carried the libm chain (C3: 6 waves 109.9 ms
    // per step, 7: 122.0, 5: 113.9); with k_flow split out, C3 runs 7 waves in
    // 86.7-87.2 ms, 6: 89.9-90.3, 8 (64 VGPRs, 5 spills): 101.9, 5: 96.4; the
    // heavier fs-7 fit (C4/C5) wanted 6 until its sweep ran on two streams (pool_for).
    if constexpr (W7) asm volatile("" ::: FARMS_POOL_FLOOR_7);
    else asm volatile("" ::: FARMS_POOL_FLOOR_6);
    uint64_t *s_start = s_dyn;
    uint32_t *s_row = reinterpret_cast<uint32_t *>(s_start + nbw);
    double *s_val = reinterpret_cast<double *>(s_start + nbw + nrs);
    uint8_t *s_k0 = reinterpret_cast<uint8_t *>(s_val + 4 * kPoolSlots);
    POOL_CLOCK(tk0);
    const int w = c0 + work_block();
    if (w >= c1) return;
    // the event and its fields in one 16-B load (k_pool_desc)
    const int4 d = c.qe[w];
    if (d.x < 0) return;  // invalid flow, or a halo event (pooled by its owner)
#ifdef FARMS_POOL_STAMPS
    PoolSt pool_st = {};
    {
        POOL_CLOCK(tk1);
        POOL_STAMP_ADD(0, tk1 - tk0);
        POOL_STAMP_ADD(5, 1);
    }
#endif
    const int e = d.x, ex = d.y, ey = d.z;
    const uint32_t teu = (uint32_t)d.w;
    const int buf = (c.ring0 + w / c.C2) % c.NB;  // the event's chunk's candidate buffer
    pool_event<K>(c, e, ex, ey, teu, buf, lane, (w / c.C2) * c.C2, s_start, s_row, s_val, s_k0 POOL_ST_ARG);
#ifdef FARMS_POOL_STAMPS
    if (lane == 0) {
        unsigned long long *row = g_pool_stamps + 8 * (blockIdx.x % kStampRows);
        for (int i = 0; i < 8; ++i) atomicAdd(&row[i], (unsigned long long)pool_st.v[i]);
    }
#endif
}

// ---------------------------------------------------------------------------
// Paired pooling (round 5): two valid events per wavefront, 32 lanes each.
// The fold is one exec-masked v_add_f64 per staged entry whatever the number
// of scales, so one event per wave issued ~157 fold instructions per valid
// event at C3 with 44 of 64 lanes in use; two events share each instruction
// when an event needs at most 32 lanes: quantities {L, L cos, L sin} of scales
// 1..K-1 on lanes 3 (k - 1) + q of the event's half (K <= 11: 30 lanes; lanes
// 30, 31 fold padding), the contributor counts from an integer histogram of
// the entries' smallest scales, and scale 0 -- the event's own cell, the one
// cell at distance 0 (an aliased second visit of it has d >= 1) -- from that
// entry's values (0 + v, vFlow.cpp:1005-1008: v itself).  Every per-scale sum
// is still the reference's sequence of additions: scale k's lane adds the
// entries with k0 <= k in raster order from 0 (pool_one's guarantees), so the
// records are bitwise k_pool's (tested).  The pass runs 32 candidates of each
// event per step; the events of a pair are consecutive pooled events of one
// pooling chunk in work order (k_pool_compact), so their windows overlap and
// their step counts match.
// (a 64-slot ring per event instead, read from a moving pointer so that a
// step's rest stays in place: C3 74.0 against 72.0 ms, profiles/r05_ab_s2.log)
constexpr int kPairSlots = 40;  // staged entries per event: <= 32 per step + < 8 carried
template <int K>
constexpr bool kPairPool = K >= 2 && K <= 11;
constexpr uint32_t kPairJunk = 0x1E1E1E1Eu;  // four shift bytes of 30: the half's lanes 30, 31 only
// LDS of a paired-pooling wave, per event: segment-start bitmap, row segments,
// staged {L, L cos, L sin} and shift bytes, the smallest-scale histogram, the
// own cell's entry
__host__ __device__ constexpr int pair_half_words(int bw, int rs) {
    return bw + rs + 3 * kPairSlots + kPairSlots / 8 + 8 /* hist: 16 ints */ + 4 /* own: L, Lc, Ls, flag */;
}
// The pair bitmap marks segment starts over the first kPairBitPos flattened
// window positions only (17 words instead of 161 at maxWindow 50: 4.1 KB of
// LDS per wave instead of 6.4, C3 72.2 -> 70.0 ms per step on the timing
// build, profiles/r05_ab_s3.log).  An event whose window holds more candidates
// (none at C3: at most 899, the scan-width tail of the bench line) is pooled
// by k_pool_ovf after the launch, one event per wave with the full bitmap.
constexpr int kPairBitPos = 1024;
__host__ __device__ constexpr int pair_bw(int bw) { return bw > kPairBitPos / 64 + 1 ? kPairBitPos / 64 + 1 : bw; }

// Ordered compaction of each pooling chunk's pooled events (valid flow, owned
// column) to the front of its work-order positions: qe[cs + r] = the r-th one's
// {event, x, y, t}, nv[ch] = their number.  One 256-thread block per chunk.
__global__ __launch_bounds__(256) void k_pool_compact(Ctx c, int ch0, int ch1, int32_t *nv, int *ovfn) {
    __shared__ int s_wsum[4];
    const int ch = ch0 + (int)blockIdx.x;
    if (ch >= ch1) return;
    if (blockIdx.x == 0 && threadIdx.x == 0) *ovfn = 0;  // the launch's overflow list starts empty
    const int cs = ch * c.C2, ce = min(cs + c.C2, c.n);
    const int tid = (int)threadIdx.x, lane = tid & 63, wv = tid >> 6;
    int carry = 0;
    for (int base = cs; base < ce; base += 256) {
        const int w = base + tid;
        bool ok = false;
        int4 fd = make_int4(0, 0, 0, 0);
        if (w < ce) {
            fd = c.fdesc[w];
            ok = c.valid[fd.x] && fd.y >= c.own_lo && fd.y < c.own_hi;
        }
        const uint64_t bal = __ballot(ok);
        if (lane == 0) s_wsum[wv] = (int)__popcll(bal);
        __syncthreads();
        int off = carry;
        for (int i = 0; i < wv; ++i) off += s_wsum[i];
        const int tot = s_wsum[0] + s_wsum[1] + s_wsum[2] + s_wsum[3];
        if (ok) c.qe[mbcnt64(bal, cs + off)] = fd;
        __syncthreads();  // (s_wsum is rewritten next round)
        carry += tot;
    }
    if (tid == 0) nv[ch] = carry;
}

// Inclusive prefix sum within each 32-lane half (wave_incl_scan without its
// last, half-crossing step).
__device__ __forceinline__ int half_incl_scan(int v) {
    // DPP with bound_ctrl: a lane without a source in its row reads 0, so each
    // row shift is one DPP-fused add.  Full exec mask expected.
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, true);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, true);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, true);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, true);   // row_shr:8
    const int t = __builtin_amdgcn_mov_dpp(v, 0x142, 0xF, 0xF, false);  // row_bcast:15 (rows 1, 3 from rows 0, 2)
    if ((__lane_id() & 31) >= 16) v += t;
    return v;
}

// Max within each 32-lane half (exact).
__device__ __forceinline__ double half_max(double v) {
    v = fmax(v, xch<0>(v));
    v = fmax(v, xch<1>(v));
    v = fmax(v, xch<2>(v));
    v = fmax(v, xch<3>(v));
    v = fmax(v, xch<4>(v));
    return v;
}

// pool_rows for two windows: half h builds its event's row table (rows hl,
// hl + 32, hl + 64, hl + 96) into its own LDS arrays; returns the half's
// flattened length (0 for an absent event).  MODE: the chunk buffer's slot
// layout (kSlotsGroup: k_chain's, a row segment splits where it crosses into
// the next 256-cell group; kSlotsBand: k_cand's band-contiguous slots, a
// segment splits only where the W - 1 clip carries it across a band boundary;
// kSlotsBandFlat: the same for windows that stay inside their x-rows, where
// no segment splits).
template <int MODE>
__device__ __forceinline__ int pool_rows2(const Ctx &c, int buf, int lane, bool act, int i_lo, int nrows, int j_lo,
                                          int j_hi, uint64_t *s_start, uint32_t *s_row, int &nseg) {
    const int H = c.H;
    const int WHl = (int)c.WH, OFF = c.X0 * c.H;
    const int WHs = (int)c.WHs;
    const int hl = lane & 31;
    const uint64_t hm = lane < 32 ? 0x00000000FFFFFFFFull : 0xFFFFFFFF00000000ull;
    uint32_t *const sbits = reinterpret_cast<uint32_t *>(s_start);
    {
        int nw = act ? ((nrows * (j_hi - j_lo + 1) + 63) >> 6) + 1 : 0;
        if (nw > kPairBitPos / 64 + 1) nw = kPairBitPos / 64 + 1;
        for (int i = hl; i < nw; i += 32) s_start[i] = 0;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    constexpr int NB = 4;  // row batches: 2M + 1 <= 127 rows
    const BmWord *bwb = c.bw_ring + (int64_t)buf * c.nwords;
    const int wmax = (int)c.nwords - 1;
    int lo_[NB], hi0_[NB], hi1_[NB], gb_[NB];
    bool has_[NB], str_[NB];
    uint64_t bA[NB], bB[NB], bC[NB];
    uint32_t oA[NB], oB[NB], oC[NB];
    const int base0 = (i_lo + hl) * H;  // (rows past the window: addresses clamped below, has_ false)
#pragma unroll
    for (int hh = 0; hh < NB; ++hh) {
        const int r = hl + 32 * hh;
        const int base = base0 + 32 * hh * H;
        int l1 = base + j_hi;
        if (l1 > WHs - 1) l1 = WHs - 1;  // past the end of the sensor: no contribution
        int l0 = base + j_lo - OFF;
        l1 -= OFF;
        if (l0 < 0) l0 = 0;               // outside the stored region: never visited
        if (l1 > WHl - 1) l1 = WHl - 1;
        has_[hh] = act && r < nrows && l0 <= l1;
        int gb;
        if constexpr (MODE == kSlotsGroup) {
            gb = l1 & ~(kGroupCells - 1);
            str_[hh] = has_[hh] && l0 < gb;
        } else if constexpr (MODE == kSlotsBand) {
            gb = band_split(c, i_lo + r);  // the first band start past l0
            str_[hh] = has_[hh] && gb <= l1;
        } else {
            gb = 0;
            str_[hh] = false;
        }
        lo_[hh] = l0; gb_[hh] = gb;
        hi0_[hh] = str_[hh] ? gb - 1 : l1;
        hi1_[hh] = l1;
        // word indices clamped for the loads only (a row without cells keeps has_
        // false): l0 >= 0 here, and a negative l1 wraps to wmax as unsigned
        const uint32_t wa = min((uint32_t)l0 >> 6, (uint32_t)wmax), wc = min((uint32_t)l1 >> 6, (uint32_t)wmax);
        const BmWord A = at32(bwb, wa), C = at32(bwb, wc);
        bA[hh] = A.bm; oA[hh] = A.wo;
        bC[hh] = C.bm; oC[hh] = C.wo;
        if constexpr (MODE != kSlotsBandFlat) {
            const uint32_t wb = min((uint32_t)hi0_[hh] >> 6, (uint32_t)wmax);
            const BmWord B = at32(bwb, wb);
            bB[hh] = B.bm; oB[hh] = B.wo;
        } else {
            bB[hh] = 0; oB[hh] = 0;
        }
    }
    int carry = 0, nz = 0;
#pragma unroll
    for (int hh = 0; hh < NB; ++hh) {
        const int r = hl + 32 * hh;
        const int lo = (int)(oA[hh] + (uint32_t)__popcll(bA[hh] & ((1ull << (lo_[hh] & 63)) - 1)));
        const int h1 = (int)(oC[hh] + (uint32_t)__popcll(bC[hh] & ((2ull << (hi1_[hh] & 63)) - 1)));
        int n0, n1;
        if constexpr (MODE == kSlotsBandFlat) {
            n0 = has_[hh] ? h1 - lo : 0;
            n1 = 0;
        } else {
            const int h0 = (int)(oB[hh] + (uint32_t)__popcll(bB[hh] & ((2ull << (hi0_[hh] & 63)) - 1)));
            n0 = has_[hh] ? h0 - lo : 0;
            n1 = str_[hh] ? h1 - gb_[hh] : 0;
        }
        const int cnt = n0 + n1;
        const int incl = half_incl_scan(cnt);
        const int start = carry + incl - cnt;
        const uint64_t b0 = __ballot(n0 > 0) & hm;
        const uint64_t b1 = MODE == kSlotsBandFlat ? 0ull : __ballot(n1 > 0) & hm;
        int idx = MODE == kSlotsBandFlat ? mbcnt64(b0, nz) : mbcnt64(b1, mbcnt64(b0, nz));
        if (n0 > 0) {
            s_row[idx++] = ((uint32_t)r << 25) | (uint32_t)(lo - start + kRowBias);
            if (start < kPairBitPos) atomicOr(&sbits[start >> 5], 1u << (start & 31));
        }
        if (n1 > 0) {
            const int st1 = start + n0;
            s_row[idx] = ((uint32_t)r << 25) | (uint32_t)(gb_[hh] - st1 + kRowBias);
            if (st1 < kPairBitPos) atomicOr(&sbits[st1 >> 5], 1u << (st1 & 31));
        }
        nz += (int)__popcll(b0) + (int)__popcll(b1);
        const int tA = __builtin_amdgcn_readlane(incl, 31), tB = __builtin_amdgcn_readlane(incl, 63);
        carry += lane < 32 ? tA : tB;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    nseg = nz;
    return carry;
}

// Fold of 8 entry slots of both events: slot u adds event A's entry on the
// lanes of A's half selected by byte u of a0:a1 (lanes >= 3 (k0 - 1) of the
// half: the scales containing the entry; 30: padding, the half's junk lanes)
// and B's likewise from b0:b1 (exec_lo, exec_hi), one v_add_f64 for both.  As
// fold8_salu: a full exec at entry (fold_exec_check), SCC clobbered, exec
// restored.
__device__ __forceinline__ void fold8_pair(double &acc, uint32_t a0, uint32_t a1, uint32_t b0, uint32_t b1,
                                           const double (&v)[8]) {
    fold_exec_check();
    uint64_t sv;
    uint32_t ta, tb;
#define FARMS_PAIR_SLOT(WA, WB, SH, V)                                                             \
    "s_lshr_b32 %[ta], %[" WA "], " SH "\n"                                                        \
    "s_lshr_b32 %[tb], %[" WB "], " SH "\n"                                                        \
    "s_lshl_b32 exec_lo, -1, %[ta]\n"                                                              \
    "s_lshl_b32 exec_hi, -1, %[tb]\n"                                                              \
    "v_add_f64 %[acc], %[acc], %[" V "]\n"
    asm volatile(
        "s_mov_b64 %[sv], exec\n"
        FARMS_PAIR_SLOT("a0", "b0", "0", "v0") FARMS_PAIR_SLOT("a0", "b0", "8", "v1")
        FARMS_PAIR_SLOT("a0", "b0", "16", "v2") FARMS_PAIR_SLOT("a0", "b0", "24", "v3")
        FARMS_PAIR_SLOT("a1", "b1", "0", "v4") FARMS_PAIR_SLOT("a1", "b1", "8", "v5")
        FARMS_PAIR_SLOT("a1", "b1", "16", "v6") FARMS_PAIR_SLOT("a1", "b1", "24", "v7")
        "s_mov_b64 exec, %[sv]\n"
        : [acc] "+v"(acc), [sv] "=&s"(sv), [ta] "=&s"(ta), [tb] "=&s"(tb)
        : [a0] "s"(a0), [a1] "s"(a1), [b0] "s"(b0), [b1] "s"(b1), [v0] "v"(v[0]), [v1] "v"(v[1]),
          [v2] "v"(v[2]), [v3] "v"(v[3]), [v4] "v"(v[4]), [v5] "v"(v[5]), [v6] "v"(v[6]), [v7] "v"(v[7])
        : "scc");
#undef FARMS_PAIR_SLOT
}

// The candidate pass and the scale choice of a pair (pool_one / pool_finish
// for two events): lanes of half h work on event h (its fields per lane).
template <int K>
__device__ __forceinline__ void pool_pair(const Ctx &c, int lane, bool act, int e, int ex, int ey, uint32_t teu,
                                          int buf, int row_i0, int total, int totA, int totB,
                                          const uint64_t *s_start, const uint32_t *s_row, double *s_val,
                                          uint8_t *s_k0, int *s_hist, double *s_own, int nseg) {
    static_assert(kPairPool<K>, "paired pooling: 3 (K - 1) <= 30 lanes per event");
    const CandHdr *chdr = c.hdr_ring + (int64_t)buf * c.cstride;
    const CandVal *cval = c.val_ring + (int64_t)buf * c.cstride;
    const int H = c.H, J = c.J;
    const int OFF = c.X0 * c.H;
    const int hl = lane & 31;
    const uint64_t hm = lane < 32 ? 0x00000000FFFFFFFFull : 0xFFFFFFFF00000000ull;
    // serial mode: the own cell is pooled with the stamp its lastEventTime
    // still holds (vFlow.cpp:790 vs :264)
    const uint32_t own_lin = c.serial ? (uint32_t)((ex - c.X0) * H + ey) : 0xFFFFFFFFu;
    const uint32_t own_tprev = c.serial ? (uint32_t)c.link[e].w : 0u;
    // this lane's fold: quantity q of scale kk (lanes 30, 31 of the half: junk)
    const int q = hl % 3;
    // the half's histogram and own entry start empty
    if (hl < 16) s_hist[hl] = 0;
    if (hl < 4) s_own[hl] = 0.0;
    double acc = 0.0;
    int ncon = 0;
    const double *const vdummy = reinterpret_cast<const double *>(c.evf + e);
    int mbase = 0;
    // flattened position f0 + hl of this half's window
    auto locate = [&](int f0, int &row, int &k) {
        const uint64_t mk = s_start[f0 >> 6];
        const int bit = (f0 & 63) + hl;
        int m = mbase + (int)__popcll(mk & ((2ull << bit) - 1)) - 1;
        if ((f0 & 63) == 32) mbase += (int)__popcll(mk);
        // a half past its window's end (or without an event) reads bitmap
        // words it never wrote: keep its segment index inside its own table
        // (its k is replaced by safe_k's anyway)
        m = m > nseg - 1 ? nseg - 1 : m;
        const uint32_t rs = s_row[m < 0 ? 0 : m];
        row = (int)(rs >> 25);
        k = f0 + hl + (int)(rs & 0x1FFFFFFu) - kRowBias;
    };
    const int tmax = totA > totB ? totA : totB;  // (wave-uniform)
    // a valid candidate index for lanes past their window's end (lane 0's or
    // lane 32's, whichever half is still scanning)
    auto safe_k = [&](int f0, int k) {
        const int kA = __builtin_amdgcn_readlane(k, 0), kB = __builtin_amdgcn_readlane(k, 32);
        return (uint32_t)(f0 < totA ? kA : kB);
    };
    int rc = 0, kc = 0;
    CandHdr hc{};
    if (tmax > 0) {
        locate(0, rc, kc);
        const uint32_t sk = safe_k(0, kc);
        hc = at32(chdr, act && hl < total ? (uint32_t)kc : sk);
    }
    uint64_t pbal = 0;
    double pv0 = 0.0, pv1 = 0.0, pv2 = 0.0;
    int pk0 = K;
    int stA = 0, stB = 0;  // (wave-uniform) staged entries not yet folded, per event
    for (int f0 = 0;; f0 += 32) {
        const bool have = f0 < tmax;  // wave-uniform
        bool con = false;
        int k0 = K;
        const double *vp = vdummy;
        if (have && act && f0 + hl < total) {
            const CandHdr &hd = hc;
            uint32_t tq;
            bool ok;
            if (hd.e1 > e) { ok = (hd.lin & kCandSnapOk) != 0; tq = hd.t_snap; vp = &cval[kc].L_snap; }
            else if (!(hd.lin & kCandMore)) { ok = (hd.lin & kCandOneOk) != 0; tq = hd.t1; vp = &cval[kc].L1; }
            else if (!(hd.lin & kCandMore2)) {
                const int2 r2 = *reinterpret_cast<const int2 *>(&cval[kc].run_lo);
                const int e2 = r2.x & 0x7FFFFFFF;
                if (e2 > e) { ok = (hd.lin & kCandOneOk) != 0; tq = hd.t1; vp = &cval[kc].L1; }
                else { ok = r2.x < 0; tq = (uint32_t)r2.y; vp = &c.evf[e2].L; }
            } else {
                const CandVal &cv = cval[kc];
                const int sev = c.P[run_search_bounds(c, cv.run_lo, cv.run_hi, e)];
                const FlowCell fe = c.evf[sev];
                ok = fe.L > 0; tq = fe.t; vp = &c.evf[sev].L;
            }
            if ((hd.lin & kCandLinMask) == own_lin) tq = own_tprev;
            const int64_t dt = (int64_t)teu - (int64_t)tq;  // |t_e - t_cell| < 500 us (vFlow.cpp:1002/1115)
            const int i = row_i0 + rc;
            const int j = (int)(hd.lin & kCandLinMask) + OFF - (int)__umul24((uint32_t)i, (uint32_t)H);
            if (ok && (uint64_t)(dt + 499) < 999u) {
                const int di = i > ex ? i - ex : ex - i, dj = j > ey ? j - ey : ey - j;
                const int d = di > dj ? di : dj;
                k0 = J == 1 ? d : (int)__umulhi((uint32_t)(d + J - 1), c.kmagic);
                con = true;
            }
        }
        if (!con) vp = vdummy;
        const double v0 = vp[0], v1 = vp[1], v2 = vp[2];
        int rn = 0, kn = 0;
        CandHdr hn = hc;
        if (f0 + 32 < tmax) {  // (wave-uniform)
            locate(f0 + 32, rn, kn);
            const uint32_t sk = safe_k(f0 + 32, kn);
            hn = at32(chdr, act && f0 + 32 + hl < total ? (uint32_t)kn : sk);
        }
        // ---- stage and fold the previous step's contributors of both events
        if (pbal) {
            const int cA = (int)__popcll(pbal & 0xFFFFFFFFull), cB = (int)__popcll(pbal >> 32);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            if ((pbal >> lane) & 1) {
                const int slot = mbcnt64(pbal & hm, lane < 32 ? stA : stB);
                s_val[3 * slot] = pv0; s_val[3 * slot + 1] = pv1; s_val[3 * slot + 2] = pv2;
                s_k0[slot] = (uint8_t)(pk0 > 0 ? 3 * (pk0 - 1) : 0);
                atomicAdd(&s_hist[pk0], 1);
                if (pk0 == 0) { s_own[0] = pv0; s_own[1] = pv1; s_own[2] = pv2; s_own[3] = 1.0; }
            }
            stA += cA;
            stB += cB;
            ncon += lane < 32 ? cA : cB;
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            const int wA = stA & ~7, wB = stB & ~7;
            const int wmaxg = wA > wB ? wA : wB;
            const uint32_t *k4p = reinterpret_cast<const uint32_t *>(s_k0);
#pragma unroll 1
            for (int r = 0; r < wmaxg; r += 8) {
                const uint32_t kw0 = k4p[r >> 2], kw1 = k4p[(r >> 2) + 1];
                double vv[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) vv[u] = s_val[3 * (r + u) + q];
                const uint32_t a0 = __builtin_amdgcn_readlane(kw0, 0), a1 = __builtin_amdgcn_readlane(kw1, 0);
                const uint32_t b0 = __builtin_amdgcn_readlane(kw0, 32), b1 = __builtin_amdgcn_readlane(kw1, 32);
                fold8_pair(acc, r < wA ? a0 : kPairJunk, r < wA ? a1 : kPairJunk, r < wB ? b0 : kPairJunk,
                           r < wB ? b1 : kPairJunk, vv);
            }
            const int rA = stA - wA, rB = stB - wB;
            // carry each event's rest (< 8) to its slots [0, rest)
            const int w_h = lane < 32 ? wA : wB, r_h = lane < 32 ? rA : rB;
            if ((wA > 0 && rA > 0) || (wB > 0 && rB > 0)) {
                double m0 = 0.0, m1 = 0.0, m2 = 0.0;
                uint8_t mk = 0;
                const bool mv = w_h > 0 && hl < r_h;
                if (mv) {
                    m0 = s_val[3 * (w_h + hl)]; m1 = s_val[3 * (w_h + hl) + 1]; m2 = s_val[3 * (w_h + hl) + 2];
                    mk = s_k0[w_h + hl];
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                __builtin_amdgcn_wave_barrier();
                if (mv) {
                    s_val[3 * hl] = m0; s_val[3 * hl + 1] = m1; s_val[3 * hl + 2] = m2;
                    s_k0[hl] = mk;
                }
            }
            stA = rA;
            stB = rB;
        }
        if (!have) break;
        pbal = __ballot(con);
        pv0 = v0; pv1 = v1; pv2 = v2;
        pk0 = k0;
        hc = hn; rc = rn; kc = kn;
    }
    if (stA > 0 || stB > 0) {  // the last groups, padded with junk entries
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const int st_h = lane < 32 ? stA : stB;
        if (hl >= st_h && hl < 8) s_k0[hl] = (uint8_t)30;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const uint32_t *k4p = reinterpret_cast<const uint32_t *>(s_k0);
        const uint32_t kw0 = k4p[0], kw1 = k4p[1];
        double vv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) vv[u] = s_val[3 * u + q];
        const uint32_t a0 = __builtin_amdgcn_readlane(kw0, 0), a1 = __builtin_amdgcn_readlane(kw1, 0);
        const uint32_t b0 = __builtin_amdgcn_readlane(kw0, 32), b1 = __builtin_amdgcn_readlane(kw1, 32);
        fold8_pair(acc, stA > 0 ? a0 : kPairJunk, stA > 0 ? a1 : kPairJunk, stB > 0 ? b0 : kPairJunk,
                   stB > 0 ? b1 : kPairJunk, vv);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // ---- the scale choice per half (vFlow.cpp:1023-1059): lane hl < K holds
    // scale hl's mean; scale 0 is the own entry alone (0 + v = v), scale k >= 1
    // lane 3 (k - 1) + q's sums; counts from the histogram (exact integers)
    const int base = lane & 32;
    const int kl = hl < K ? hl : 0;
    // counts per scale: the histogram's prefix sums over the half's lanes
    // (lane hl < K: contributors with smallest scale <= hl)
    const int pref = half_incl_scan(hl < K ? s_hist[hl] : 0);
    const int cnt = pref;
    const bool own_ok = s_own[3] != 0.0;
    const double len_k = __shfl(acc, base + 3 * (kl > 0 ? kl - 1 : 0), 64);
    const double L_k = kl == 0 ? (own_ok ? s_own[0] : 0.0) : len_k;
    const bool is_len = act && hl < K;
    const double mean = is_len && cnt > 0 ? L_k / (double)cnt : 0.0;
    const double maxv = half_max(mean);
    const uint64_t win = __ballot(is_len && mean == maxv) & hm;
    const int mi = maxv > 0 ? (int)__builtin_ctzll(win) - base : 0;
    const int miA = __builtin_amdgcn_readlane(mi, 0), miB = __builtin_amdgcn_readlane(mi, 32);
    const int cnt_mi = lane < 32 ? __builtin_amdgcn_readlane(pref, miA) : __builtin_amdgcn_readlane(pref, 32 + miB);
    const int src = base + 3 * (mi > 0 ? mi - 1 : 0);
    const double sx_s = __shfl(acc, src + 1, 64), sy_s = __shfl(acc, src + 2, 64);
    const double sx = mi == 0 ? s_own[1] : sx_s, sy = mi == 0 ? s_own[2] : sy_s;
    // lane 0 of the half takes Gx, lane 1 Gy: one division sequence for both
    if (act && hl < 2) {
        double g;
        if (maxv > 0) {
            g = (hl == 0 ? sx : sy) / (double)cnt_mi;  // vFlow.cpp:1028-1029, 1067-1075
        } else {  // vFlow.cpp:1085-1094
            const FlowCell &self = c.evf[e];
            g = hl == 0 ? self.Lc : self.Ls;
        }
        (hl == 0 ? c.r_true : c.th_true)[e] = g;  // (RTrue, ThetaTrue) by k_true_polar
        if (hl == 0) {
            c.scale[e] = maxv > 0 ? mi * J : 0;
            if (c.dbg_tc) c.dbg_tc[e] = make_int2(total, ncon);
        }
    }
}

// Two pooled events of a pooling chunk per wavefront (kPairPool): pair p of
// chunk ch takes its compacted events 2p and 2p + 1 (k_pool_compact); pairs
// past the chunk's count leave at once.  Same occupancy cap as k_pool.
template <int K, bool W7>
__global__ __launch_bounds__(64, W7 ? 7 : 6) void k_pool2(Ctx c, int ch0, int ch1, const int32_t *nv, int4 *ovf,
                                                           int *ovfn) {
    extern __shared__ __attribute__((aligned(16))) uint64_t s_dyn[];
    if constexpr (W7) asm volatile("" ::: FARMS_POOL_FLOOR_7);
    else asm volatile("" ::: FARMS_POOL_FLOOR_6);
    const int lane = threadIdx.x & 63;
    const int ppc = c.C2 >> 1;  // pair slots per chunk
    const int lb = work_block();
    const int ch = ch0 + lb / ppc, p = lb % ppc;
    if (ch >= ch1) return;
    const int cs = ch * c.C2;
    // the descriptor load goes out with the count's (clamped: a partial last
    // chunk's pair slots reach past the call's events)
    const int4 dq = c.qe[min(cs + 2 * p + (lane >> 5), c.n - 1)];
    const int cnt = nv[ch];
    if (2 * p >= cnt) return;
    const bool hasB = 2 * p + 1 < cnt;
    bool act = lane < 32 || hasB;
    // a half without an event takes event A's fields: lane 0's, by readlane.
    // (readfirstlane would read the first lane of the exec mask the compiler
    // evaluates this select under -- lane 32 when only the idle half is
    // active -- i.e. the stale descriptor past the chunk's count: an event id
    // from an earlier call or handle, whose flow the idle lanes then loaded.
    // Freshly mapped memory holds zeros, so it showed only after another
    // call or handle had used the memory: the strip steps and a test sequence
    // faulted, round 5.)
    const int4 d = act ? dq : make_int4(__builtin_amdgcn_readlane(dq.x, 0), __builtin_amdgcn_readlane(dq.y, 0),
                                        __builtin_amdgcn_readlane(dq.z, 0), __builtin_amdgcn_readlane(dq.w, 0));
    const int e = d.x, ex = d.y, ey = d.z;
    const uint32_t teu = (uint32_t)d.w;
    const int buf = (c.ring0 + ch) % c.NB;  // the pair's chunk's candidate buffer
    // this half's LDS
    const int hw = pair_half_words(pair_bw(c.pool_bw), c.pool_rs);
    uint64_t *s_start = s_dyn + (lane >= 32 ? hw : 0);
    const int bwp = pair_bw(c.pool_bw);
    uint32_t *s_row = reinterpret_cast<uint32_t *>(s_start + bwp);
    double *s_val = reinterpret_cast<double *>(s_start + bwp + c.pool_rs);
    uint8_t *s_k0 = reinterpret_cast<uint8_t *>(s_val + 3 * kPairSlots);
    int *s_hist = reinterpret_cast<int *>(s_k0 + kPairSlots);
    double *s_own = reinterpret_cast<double *>(s_hist + 16);
    const int W = c.W, M = c.M;
    const int i_lo = ex - M < 0 ? 0 : ex - M, i_hi = ex + M > W - 1 ? W - 1 : ex + M;
    const int j_lo = ey - M < 0 ? 0 : ey - M, j_hi = ey + M > W - 1 ? W - 1 : ey + M;
    int nseg, total;
    if (!c.band_slots) {
        total = pool_rows2<kSlotsGroup>(c, buf, lane, act, i_lo, i_hi - i_lo + 1, j_lo, j_hi, s_start, s_row, nseg);
    } else if (__ballot(act && j_hi >= c.H)) {  // a window clipped at W - 1 past its x-row (W > H): wave-uniform
        total = pool_rows2<kSlotsBand>(c, buf, lane, act, i_lo, i_hi - i_lo + 1, j_lo, j_hi, s_start, s_row, nseg);
    } else {
        total = pool_rows2<kSlotsBandFlat>(c, buf, lane, act, i_lo, i_hi - i_lo + 1, j_lo, j_hi, s_start, s_row, nseg);
    }
    if (act && total > kPairBitPos) {  // past the bitmap: to the overflow list, pooled by k_pool_ovf
        if ((lane & 31) == 0) ovf[atomicAdd(ovfn, 1)] = d;
        act = false;
        total = 0;
        nseg = 0;
    }
    const int totA = __builtin_amdgcn_readlane(total, 0), totB = __builtin_amdgcn_readlane(total, 32);
    pool_pair<K>(c, lane, act, e, ex, ey, teu, buf, i_lo, total, totA, totB, s_start, s_row, s_val, s_k0, s_hist,
                 s_own, nseg);
}

// The events of one k_pool2 launch whose windows held more than kPairBitPos
// candidates (ovf[0, *ovfn), their descriptors), one event per wave as k_pool
// with the full bitmap, on the pooling stream right after the launch.  A fixed
// grid that strides over the list: it leaves at once when the list is empty.
constexpr int kPoolOvfBlocks = 64;
template <int K, bool W7>
__global__ __launch_bounds__(64) void k_pool_ovf(Ctx c, const int4 *ovf, const int *ovfn) {
    extern __shared__ __attribute__((aligned(16))) uint64_t s_dyn[];
    if constexpr (W7) asm volatile("" ::: FARMS_POOL_FLOOR_7);
    else asm volatile("" ::: FARMS_POOL_FLOOR_6);
    const int cnt = *ovfn;
    const int lane = threadIdx.x & 63;
    uint64_t *s_start = s_dyn;
    uint32_t *s_row = reinterpret_cast<uint32_t *>(s_start + c.pool_bw);
    double *s_val = reinterpret_cast<double *>(s_start + c.pool_bw + c.pool_rs);
    uint8_t *s_k0 = reinterpret_cast<uint8_t *>(s_val + 4 * kPoolSlots);
    for (int i = (int)blockIdx.x; i < cnt; i += (int)gridDim.x) {
        const int4 d = ovf[i];
        const int e = d.x, ch = e / c.C2;
        const int buf = (c.ring0 + ch) % c.NB;
#ifdef FARMS_POOL_STAMPS
        PoolSt pool_st = {};
#endif
        pool_event<K>(c, e, d.y, d.z, (uint32_t)d.w, buf, lane, ch * c.C2, s_start, s_row, s_val, s_k0 POOL_ST_ARG);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

// Global flow vector -> record (vFlow.cpp:365-366) for every pooled (valid,
// owned) event: k_pool leaves (Gx, Gy) in the r_true / theta_true columns.
__global__ void k_true_polar(Ctx c, int e0, int e1) {
    const int e = e0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= e1 || !c.valid[e]) return;
    const int x = c.x[e];
    if (x < c.own_lo || x >= c.own_hi) return;
    const double gx = c.r_true[e], gy = c.th_true[e];
    c.r_true[e] = sqrt(gy * gy + gx * gx);
    c.th_true[e] = F_ATAN2(gy, gx);
}

// ---------------------------------------------------------------------------
// x-strips with a flow-halo exchange (multi-GPU): the local flows
// {L, L cos(theta), L sin(theta)} of listed events out of / into evf.  An
// imported flow takes the local event's stamp; validity is L > 0 (the gate's
// L = 0 for an invalid event, vFlow.cpp:398-402).
// An index outside the fit's events [0, n) is skipped (its slot / nothing is
// written) and counted in *bad: the synchronous calls report it.
__global__ void k_export_flows(const FlowCell *evf, const int32_t *idx, int count, int n, double *out, int *bad) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const int e = idx[i];
    if (e < 0 || e >= n) { atomicAdd(bad, 1); return; }
    const FlowCell f = evf[e];
    out[3 * (int64_t)i] = f.L;
    out[3 * (int64_t)i + 1] = f.Lc;
    out[3 * (int64_t)i + 2] = f.Ls;
}

__global__ void k_import_flows(Ctx c, const int32_t *idx, int count, const double *in, int *bad) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const int e = idx[i];
    if (e < 0 || e >= c.n) { atomicAdd(bad, 1); return; }
    FlowCell f;
    f.L = in[3 * (int64_t)i];
    f.Lc = in[3 * (int64_t)i + 1];
    f.Ls = in[3 * (int64_t)i + 2];
    f.t = c.t[e];
    f.pad = 0;
    c.evf[e] = f;
    c.valid[e] = f.L > 0 ? 1 : 0;
}

// ---------------------------------------------------------------------------
// Temporal segments (multi-GPU): the SAE a segment starts from.
// Last event index per pixel (x-major, whole sensor), then its stamp.
__global__ void k_last_index(const int32_t *x, const int32_t *y, int e0, int e1, int W, int H, int32_t *last) {
    const int e = e0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= e1) return;
    const int ex = x[e], ey = y[e];
    if (ex < 0 || ex >= W || ey < 0 || ey >= H) return;  // rejected by farms_process* anyway
    atomicMax(&last[(int64_t)ex * H + ey], e);
}

// The same without scattered atomics (round 5: 50M device-scope atomicMax'es,
// one lane per address, took 2.0 ms): the events bucketed by pixel tile
// (kLastTile pixels) in two passes over blocks of kLastBlock events -- counts
// per tile in LDS, one reservation per (block, tile), slots by LDS cursors --
// then one workgroup per tile keeps its pixels' last event in LDS (for the
// head [0, n_head) and for all events) and writes both stamp surfaces.
// (blocks of 131,072 events: each block's per-tile counts go to global memory as
// one-lane atomics, ≈900 per block at 1280x720, which at 16,384 events per
// block made the two passes 1.4 ms of the call)
constexpr int kLastTile = 1024, kLastBlock = 131072, kLastMaxTiles = 4096;
__device__ __forceinline__ int last_pix(const int32_t *x, const int32_t *y, int e, int W, int H) {
    const int ex = x[e], ey = y[e];
    return (ex < 0 || ex >= W || ey < 0 || ey >= H) ? -1 : ex * H + ey;  // (rejected by farms_process* anyway)
}
__global__ __launch_bounds__(1024) void k_last_bucket(const int32_t *x, const int32_t *y, int n, int W, int H,
                                                      int ntiles, int *tcount, int *tcur, int2 *bucket, int place) {
    // a wave reads 64 consecutive events (coalesced); the lanes of one run of
    // equal tiles make one LDS atomic, by the run's first lane.  (Measured: one
    // LDS atomic per distinct tile of the wave, 3.3 ms a pass -- a wave's
    // events span tens of tiles; a run of events per thread, 9 ms -- its loads
    // uncoalesced.  What is left is the bucket pass's scattered 8-B writes.)
    __shared__ int s_cnt[kLastMaxTiles], s_base[kLastMaxTiles];
    for (int i = threadIdx.x; i < ntiles; i += blockDim.x) s_cnt[i] = 0;
    __syncthreads();
    const int lane = (int)threadIdx.x & 63;
    const int e0 = blockIdx.x * kLastBlock, e1 = min(e0 + kLastBlock, n);
    // per 64 events (their pixels q, -1: none): tile, the run heads' mask,
    // this lane's head and, on a head, its run's length
    auto runs = [&](int q, int &tl, int &head, int &len) {
        tl = q < 0 ? -1 : q / kLastTile;
        const int prev = __shfl_up(tl, 1, 64);
        const uint64_t heads = __ballot(tl >= 0 && (lane == 0 || prev != tl));
        const uint64_t upto = heads & (lane == 63 ? ~0ull : ((2ull << lane) - 1));
        head = upto ? 63 - __clzll(upto) : 0;
        // a head's run ends at the next head or at the first lane without a tile
        const uint64_t none = __ballot(tl < 0);
        const uint64_t stop = lane == 63 ? 0ull : (heads | none) >> (lane + 1);
        len = stop ? __builtin_ctzll(stop) + 1 : 64 - lane;
    };
    for (int b = e0; b < e1; b += 4 * (int)blockDim.x) {
        int qq[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {  // four wave-batches' loads in flight together
            const int e = b + u * (int)blockDim.x + (int)threadIdx.x;
            qq[u] = e < e1 ? last_pix(x, y, e, W, H) : -1;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            int tl, head, len;
            runs(qq[u], tl, head, len);
            if (tl >= 0 && head == lane) atomicAdd(&s_cnt[tl], len);
        }
    }
    __syncthreads();
    if (!place) {  // pass 1: counts per tile
        for (int i = threadIdx.x; i < ntiles; i += blockDim.x)
            if (s_cnt[i]) atomicAdd(&tcount[i], s_cnt[i]);
        return;
    }
    // pass 2: this block's range of each tile's bucket, then each run's slots
    for (int i = threadIdx.x; i < ntiles; i += blockDim.x) {
        s_base[i] = s_cnt[i] ? atomicAdd(&tcur[i], s_cnt[i]) : 0;
        s_cnt[i] = 0;
    }
    __syncthreads();
    for (int b = e0; b < e1; b += 4 * (int)blockDim.x) {
        int qq[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = b + u * (int)blockDim.x + (int)threadIdx.x;
            qq[u] = e < e1 ? last_pix(x, y, e, W, H) : -1;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = b + u * (int)blockDim.x + (int)threadIdx.x;
            int tl, head, len;
            runs(qq[u], tl, head, len);
            int base = 0;
            if (tl >= 0 && head == lane) base = s_base[tl] + atomicAdd(&s_cnt[tl], len);
            base = __shfl(base, head, 64);
            if (tl >= 0) bucket[base + (lane - head)] = make_int2(e, qq[u] - tl * kLastTile);
        }
    }
}

// tile offsets: tcur = exclusive prefix of tcount (one block; ntiles <= kLastMaxTiles)
__global__ __launch_bounds__(1024) void k_last_offsets(const int *tcount, int ntiles, int *toff, int *tcur) {
    __shared__ int s_sum[1024];
    const int per = (ntiles + 1023) / 1024, i0 = threadIdx.x * per;
    int v = 0;
    for (int i = i0; i < min(i0 + per, ntiles); ++i) v += tcount[i];
    s_sum[threadIdx.x] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        int a = 0;
        for (int i = 0; i < 1024; ++i) { const int c = s_sum[i]; s_sum[i] = a; a += c; }
    }
    __syncthreads();
    int a = s_sum[threadIdx.x];
    for (int i = i0; i < min(i0 + per, ntiles); ++i) { toff[i] = a; tcur[i] = a; a += tcount[i]; }
    if (threadIdx.x == 1023) toff[ntiles] = a;
}
__global__ __launch_bounds__(256) void k_last_tile(const int2 *bucket, const int *toff, int n_head, const uint32_t *t,
                                                   int64_t WH, int64_t *head, int64_t *full) {
    __shared__ int s_head[kLastTile], s_full[kLastTile];
    for (int i = threadIdx.x; i < kLastTile; i += blockDim.x) { s_head[i] = -1; s_full[i] = -1; }
    __syncthreads();
    const int tl = blockIdx.x;
    for (int i = toff[tl] + (int)threadIdx.x; i < toff[tl + 1]; i += blockDim.x) {
        const int2 b = bucket[i];
        atomicMax(&s_full[b.y], b.x);
        if (b.x < n_head) atomicMax(&s_head[b.y], b.x);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kLastTile; i += blockDim.x) {
        const int64_t q = (int64_t)tl * kLastTile + i;
        if (q >= WH) break;
        const int ef = s_full[i], eh = s_head[i];
        full[q] = ef >= 0 ? (int64_t)t[ef] : int64_t(-1);
        if (head) head[q] = eh >= 0 ? (int64_t)t[eh] : int64_t(-1);
    }
}

__global__ void k_last_stamp(const int32_t *last, const uint32_t *t, int64_t WH, int64_t *out) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= WH) return;
    const int e = last[q];
    out[q] = e >= 0 ? (int64_t)t[e] : int64_t(-1);
}

// out[q] = the stamp of the last array (in order) that visited q, -1 if none.
__global__ void k_merge_stamps(const int64_t *in, int count, int64_t WH, int64_t *out) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= WH) return;
    int64_t v = -1;
    for (int i = 0; i < count; ++i) {
        const int64_t s = in[(int64_t)i * WH + q];
        v = s >= 0 ? s : v;
    }
    out[q] = v;
}

// SAE snapshot of the stored region <- whole-sensor stamps (-1: never visited).
__global__ void k_seed_sae(Ctx c, const int64_t *stamp) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= c.WH) return;
    const int64_t s = stamp[q + (int64_t)c.X0 * c.H];
    SaeHead hd{};
    hd.w = s >= 0 ? kHeadVisited : 0u;  // not touched
    hd.tsnap = s >= 0 ? (uint32_t)s : 0u;
    c.cells.head[q] = hd;  // both SAE buffers
    c.cells.head[q + c.WH + 1] = hd;  // (buffer 1 follows buffer 0's guard head)
}

// lastEventTime surface for farms_get_last_event_time: stamp of the latest
// event at each pixel, 0 when never visited (vFlow.cpp:66,264,407).
__global__ void k_last_time(const SaeHead *cells, int64_t WH, double *out) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= WH) return;
    const SaeHead s = cells[q];
    out[q] = (s.w & kHeadVisited) ? (double)s.tsnap : 0.0;
}

// Algorithmic-work counters for the roofline: U_loc per event,
// U_pool per valid event, valid count.  Grid-stride, one atomic per block.
__global__ void k_stats(Ctx c) {
    unsigned long long nv = 0, usae = 0, upool = 0, ncand = 0, ncon = 0, nown = 0, nwide = 0;
    unsigned int smax = 0;
    const int fr = c.fr;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < c.n;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int x = c.x[e], y = c.y[e];
        const int u0 = max(0, x - 2 * fr), u1 = min(c.W - 1, x + 2 * fr);
        const int v0 = max(0, y - 2 * fr), v1 = min(c.H - 1, y + 2 * fr);
        usae += (unsigned long long)(u1 - u0 + 1) * (unsigned long long)(v1 - v0 + 1);
        const bool own = x >= c.own_lo && x < c.own_hi;
        nown += own;
        if (c.valid[e] && own) {
            ++nv;
            if (c.dbg_tc) {
                const int2 tc = c.dbg_tc[e];
                ncand += (unsigned)tc.x; ncon += (unsigned)tc.y;
                nwide += tc.x > 1024;
                smax = max(smax, (unsigned)tc.x);
            }
            const int i_lo = max(0, x - c.M), i_hi = min(c.W - 1, x + c.M);
            const int j_lo = max(0, y - c.M), j_hi = min(c.W - 1, y + c.M);
            for (int i = i_lo; i <= i_hi; ++i) {
                const int64_t l0 = (int64_t)i * c.H + j_lo;
                int64_t l1 = (int64_t)i * c.H + j_hi;
                if (l1 > c.WHs - 1) l1 = c.WHs - 1;
                if (l1 >= l0) upool += (unsigned long long)(l1 - l0 + 1);
            }
        }
    }
    constexpr int NC = 8;  // sums, then the max (slot 7)
    __shared__ unsigned long long s[NC][256];
    s[0][threadIdx.x] = nv; s[1][threadIdx.x] = usae; s[2][threadIdx.x] = upool;
    s[3][threadIdx.x] = ncand; s[4][threadIdx.x] = ncon; s[5][threadIdx.x] = nown;
    s[6][threadIdx.x] = nwide; s[7][threadIdx.x] = smax;
    __syncthreads();
    for (int st = blockDim.x / 2; st > 0; st >>= 1) {
        if ((int)threadIdx.x < st) {
            for (int r = 0; r < NC - 1; ++r) s[r][threadIdx.x] += s[r][threadIdx.x + st];
            s[7][threadIdx.x] = max(s[7][threadIdx.x], s[7][threadIdx.x + st]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        for (int r = 0; r < NC - 1; ++r) atomicAdd(&c.counters[r], s[r][0]);
        atomicMax(&c.counters[7], s[7][0]);
    }
}

inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

}  // namespace

// ===========================================================================
// handle

// Per-call workspace.  Two sets: the host-array path pipelines a call in
// sub-batches, and sub-batch b + 1's upload and prep (set (b+1) % 2) run while
// sub-batch b's sweeps still read set b % 2.  The two-phase strip calls
// alternate too: the fit of sub-batch b+2 waits for the pooling of b (a third
// set that let it run ahead measured slower: its fit waves crowd the pooling,
// DESIGN.md §6).
struct Work {
    int64_t cap = 0;
    uint32_t *pix = nullptr, *skey = nullptr;
    int32_t *iota = nullptr, *P = nullptr;
    int2 *PT = nullptr;
    int4 *link = nullptr;
    int32_t *Q = nullptr;
    int4 *qe = nullptr, *fdesc = nullptr;
    double2 *plane = nullptr;
    uint32_t *wkey = nullptr, *wkey_sorted = nullptr;
    uint8_t *valid = nullptr;
    FlowCell *evf = nullptr;
    int2 *dbg_tc = nullptr;
    uint32_t *ctmin = nullptr, *ctmax = nullptr;
    uint32_t *cpmax = nullptr;                 // k_cand plan: prefix maximum of ctmax
    int32_t *cbk = nullptr;                    // k_cand plan: first chunk reaching each chunk's kill window
    int32_t *bstart = nullptr;                 // k_cand: per chunk, the work-order start of each column band
    int32_t *nv = nullptr;                     // paired pooling: per chunk, its pooled events (k_pool_compact)
    int4 *ovf = nullptr;                       // paired pooling: events past the pair bitmap (k_pool_ovf)
    int *ovfn = nullptr;                       // ... their number per super-chunk (list at the super-chunk's first event)
    int4 *s2x = nullptr;                       // k_cand_export: per chunk, its S2 sources
    int32_t *s2b = nullptr;                    // ... and their column bands' starts
    void *cub_tmp = nullptr;
    size_t cub_bytes = 0;
    int32_t *pcur = nullptr, *pend = nullptr;  // per cell: the call's pooling-chain cursor / last run position
    int4 *slist = nullptr;                     // k_cand: the call-start snapshot list (<= kCandMaxList)
    int *cinfo = nullptr;                      // k_cand: the call's plan (kCiWords)
    hipEvent_t plan_ev = nullptr;              // the plan's reach (kCiMaxBack) is in the handle's pinned word
    std::vector<hipEvent_t> sync_ev;           // dependency events of a call (no timing)
    hipEvent_t done = nullptr;                 // recorded after every use of the set by an asynchronous call
    hipEvent_t ready = nullptr;                // two-phase calls: the fits and the imported flows are in place
    bool ready_host = false;                   // ... and the host has seen `ready` complete (export / import synced F)
    hipEvent_t fend = nullptr;                 // asynchronous calls: stream F's last work of the call
    bool busy = false;                         // `done` recorded and the set not yet reused
};

struct farms_handle {
    farms_params prm;
    int W = 0, H = 0, fr = 0, J = 0, M = 0, K = 0;
    int64_t WH = 0;  // stored cells (region)
    int X0 = 0, WR = 0, own_lo = 0, own_hi = 0;
    int fit_chunk = kDefaultFitChunk, pool_chunk = kDefaultPoolChunk;
    hipStream_t stream = nullptr;
    // persistent surfaces (x-major, W*H cells)
    SaeHead *sae_head = nullptr;  // two buffers of WH + 1 heads (fit-chunk parity; the last one a zero guard), then
    SaeTail *sae_tail = nullptr;  // two of WH + 1 tails
    int64_t *ftime = nullptr;
    FlowCell *fsnap = nullptr;
    // ring of per-chunk candidate buffers (NB = 3 x pool_batch + 1), indexed by
    // the chunk's number since the last reset (calls continue the ring): the
    // candidate build of super-chunk S overwrites only buffers of S - 3
    int pool_batch = kDefaultPoolBatch, NB = 3 * kDefaultPoolBatch + 1;
    BmWord *bw_ring = nullptr;
    int nblk = 0;
    int64_t cstride = 0;
    CandHdr *hdr_ring = nullptr;
    CandVal *val_ring = nullptr;
    int64_t nwords = 0;
    int nbands = 1, bandc = 0;   // k_cand: column bands, columns per band
    bool cand_ok = true;          // the bands fit k_cand's LDS bitmap (else every call takes k_chain)
    int32_t *cscr = nullptr;      // k_cand: candidate items per (chunk of a launch, slice)
    int cand_last = -1;           // the last pooling call's candidate build: 1 k_cand, 0 k_chain
    int *plan_pin = nullptr;      // pinned: kCiMaxBack of each workspace set's last prep
    int64_t chunk_base = 0, super_base = 0;  // pooling chunks / super-chunks enqueued since the last reset
    hipEvent_t gpool[4] = {};                // pooling done of the last super-chunks (by number % 4)
    hipEvent_t chain_end = nullptr;          // the last call's candidate chain done
    hipEvent_t ex_ev = nullptr;              // farms_export_flows_async: its gather done (stream F)
    void *last_buf = nullptr;                // farms_last_stamps: tile counts and event buckets (grown on demand)
    size_t last_cap = 0;
    int ex_set = -1;                         // ... the workspace set it read (-1: none pending)
    hipStream_t polar_stream = nullptr;      // where the last k_true_polar was enqueued, and for which
    int64_t polar_super = -1;                // super-chunk (record_pool_done checks them)
    hipStream_t s_chain = nullptr, s_pool = nullptr;  // candidate-building chain, pooling kernels
    uint32_t seq = 0;
    // workspace sets: device and host calls use sets 0 and 1; the two-phase
    // calls rotate over all three, so that the fit of sub-batch b + 2 does not
    // wait for the pooling of b (which held the x-strip pipeline's fits and
    // poolings to taking turns)
    Work ws[3];
    // two-phase calls (farms_fit_device / farms_pool_device): the fits not yet
    // pooled, oldest first (at most two: the fit of sub-batch b+1 may be issued
    // before the pooling of b), each on its own workspace set
    struct Phase {
        const int32_t *x, *y, *p;
        const uint32_t *t;
        int64_t n;
        farms_records out;
        int set;
    };
    Phase ph[2] = {};
    int ph_count = 0;
    uint32_t ph_seq = 0;  // fits issued: the next one's workspace set is ph_seq % 3
    int64_t first_q = -1;       // serial mode: the first line's cell and stamp (farms_serial_first)
    uint32_t first_t = 0;
    bool fresh = true;          // no event since create / reset (farms_serial_first's precondition)
    int tile_bits = 0;
    int tile_shift = 3;       // work-order tile: 2^tile_shift square
    int *err = nullptr;       // device words: [0] range check, [1] k_prep, [2] export / [3] import index check, [4] async import
    int *err_pin = nullptr;   // pinned host copies of those words ([5]: the range check's)
    hipEvent_t val_ev = nullptr;  // the range check's result in err_pin[5] (s_copy)
    bool val_pending = false;     // ... not yet looked at: before the call's first fit (check_valid)
    unsigned long long *counters = nullptr;
    bool profiling = false;  // kernel timing events
    bool counting = false;   // work counters (k_stats, per-event candidate counts)
    bool fit_events = false;  // timing events around every fit launch too
    // FARMS_POISON=1 (test aid): before every call the per-event workspace the
    // call must write before it reads it -- descriptors, links, planes, flows,
    // accepted flags, the overflow list -- and, before each super-chunk's
    // candidate build, the ring buffers it is about to fill start out as 0x7F
    // bytes (event ids and slot indices ~2^31: any read of a word the call has
    // not written goes far out of range instead of finding an earlier call's
    // data, which fresh allocations hide behind zeros)
    bool poison = false;
    // Profiling across calls (farms_get_stats reports the calls since the last
    // reset): each call records timing brackets -- its phases and its kernel
    // launches -- on the streams that run them, synchronous or not; they are
    // read (and their events recycled) when the stats are asked for, so that
    // the asynchronous sub-batches of a pipelined step are counted too.
    struct Bracket {
        hipEvent_t a, b;
        int kind;  // kBr* below
    };
    std::vector<Bracket> brk;
    std::vector<hipEvent_t> ev_free;  // timing events ready for reuse
    farms_stats acc{};                // totals of the brackets read so far, launch counts, counters
    bool counters_dirty = false;      // k_stats ran since the counters were last read
    // host-array path (farms_process): pinned staging of inputs (16 B/event)
    // and records (52 B/event, or 68 with the x/y/t/p echo), an upload and a
    // download stream, one completion event per pooling super-chunk, one per
    // sub-batch upload
    uint8_t *pin_in = nullptr, *pin_out = nullptr;
    int64_t pin_cap = 0;
    // the call's device copies of the inputs and its device records, whole-call
    // sized (sub-batches are slices): a workspace set's reuse never waits for
    // an upload or a download
    int32_t *io_x = nullptr, *io_y = nullptr, *io_t = nullptr, *io_p = nullptr;  // (t as its bits)
    double *io_rec[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    int32_t *io_scale = nullptr;
    int64_t io_cap = 0;
    hipStream_t s_copy = nullptr;  // farms_process's uploads and record downloads (one stream: -3 ms at C3)
    std::vector<hipEvent_t> copy_ev;
    std::vector<hipEvent_t> final_ev;  // per super-chunk of a farms_process call: its records are final
    std::vector<hipEvent_t> up_ev;  // per sub-batch of a farms_process call: its upload landed
};

namespace {

template <typename T>
int dalloc(T **ptr, size_t count) {
    HIPCHK(hipMalloc((void **)ptr, sizeof(T) * (count ? count : 1)));
    return FARMS_OK;
}

template <typename T>
void dfree(T *&p) {
    if (p) (void)hipFree((void *)p);
    p = nullptr;
}

void free_workspace(Work &w) {
    dfree(w.pix); dfree(w.skey);
    dfree(w.iota); dfree(w.P); dfree(w.PT); dfree(w.link);
    dfree(w.Q); dfree(w.qe); dfree(w.fdesc); dfree(w.plane); dfree(w.wkey); dfree(w.wkey_sorted);
    dfree(w.valid); dfree(w.evf); dfree(w.dbg_tc); dfree(w.ctmin); dfree(w.ctmax);
    dfree(w.cpmax); dfree(w.cbk); dfree(w.bstart); dfree(w.nv); dfree(w.s2x); dfree(w.s2b); dfree(w.ovf); dfree(w.ovfn);
    dfree(w.cub_tmp);
    w.cub_bytes = 0;
    w.cap = 0;
}

int end_bit_for(int64_t WH) {
    int b = 1;
    while ((int64_t(1) << b) < WH) ++b;
    return b;
}

// Every stream of the handle idle (nothing of an asynchronous call in flight).
int sync_all(farms_handle *h) {
    for (hipStream_t s : {h->stream, h->s_chain, h->s_pool, h->s_copy})
        if (s) HIPCHK(hipStreamSynchronize(s));
    for (Work &w : h->ws) w.busy = false;
    return FARMS_OK;
}

// The pixel sort of a call's events (stable, by pixel id over end_bit bits):
// rocPRIM's onesweep with 10 bits per pass, two passes for a 1280x720 sensor's
// 20-bit ids where hipCUB's gfx950 default (8 bits) takes three (C3 66.4 ->
// 66.1, C2 2.90 -> 2.85 ms, same bits; 11 bits: 66.8,
// profiles/r06_ab_sort_bits.log).  (The 1,024-thread blocks rank with
// per-wave counters, `match`: the default per-thread ones need 2 MB of LDS at
// 10 bits.)
hipError_t pixel_sort(void *tmp, size_t &bytes, const uint32_t *kin, uint32_t *kout, const int32_t *vin, int32_t *vout,
                      int n, int end_bit, hipStream_t s) {
    using Cfg = rocprim::radix_sort_config<
        rocprim::default_config, rocprim::default_config,
        rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 8>, rocprim::kernel_config<1024, 8>, 10,
                                            rocprim::block_radix_rank_algorithm::match>>;
    return rocprim::radix_sort_pairs<Cfg>(tmp, bytes, kin, kout, vin, vout, n, 0u, (unsigned)end_bit, s);
}

int ensure_capacity(farms_handle *h, Work &w, int64_t n) {
    if (n <= w.cap) return FARMS_OK;
    int rc = sync_all(h);  // the set may still be read by an earlier call
    if (rc) return rc;
    free_workspace(w);
    const int64_t cap = n;
    const int64_t nch = (cap + h->pool_chunk - 1) / h->pool_chunk;
    if ((rc = dalloc(&w.pix, cap)) || (rc = dalloc(&w.skey, cap)) ||
        (rc = dalloc(&w.iota, cap)) || (rc = dalloc(&w.P, cap)) || (rc = dalloc(&w.PT, cap)) ||
        (rc = dalloc(&w.link, cap)) || (rc = dalloc(&w.Q, cap)) || (rc = dalloc(&w.qe, cap)) || (rc = dalloc(&w.fdesc, cap)) ||
        (rc = dalloc(&w.plane, cap)) || (rc = dalloc(&w.wkey, cap)) || (rc = dalloc(&w.wkey_sorted, cap)) ||
        (rc = dalloc(&w.valid, cap)) || (rc = dalloc(&w.evf, cap)) || (rc = dalloc(&w.dbg_tc, cap)) ||
        (rc = dalloc(&w.ctmin, nch)) || (rc = dalloc(&w.ctmax, nch)) || (rc = dalloc(&w.cpmax, nch)) ||
        (rc = dalloc(&w.cbk, nch)) || (rc = dalloc(&w.bstart, nch * (h->nbands + 1))) || (rc = dalloc(&w.nv, nch)) ||
        (rc = dalloc(&w.ovf, cap)) || (rc = dalloc(&w.ovfn, nch)) ||
        (rc = dalloc(&w.s2x, cap)) || (rc = dalloc(&w.s2b, nch * (h->nbands + 1)))) {
        free_workspace(w);
        return rc;
    }
    size_t bytes = 0, bytes2 = 0;
    HIPCHK(pixel_sort(nullptr, bytes, w.pix, w.skey, w.iota, w.P, (int)cap, end_bit_for(h->WH), h->stream));
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes2, w.wkey, w.wkey_sorted, w.iota, w.Q, (int)cap, 0,
                                              32, h->stream));
    bytes = std::max(bytes, bytes2);
    if ((rc = dalloc((uint8_t **)&w.cub_tmp, bytes))) { free_workspace(w); return rc; }
    w.cub_bytes = bytes;
    w.cap = cap;
    return FARMS_OK;
}

// Timing brackets (farms_handle::brk).
enum { kBrPrep = 0, kBrFitSweep, kBrPoolSweep, kBrFitKernel, kBrPoolKernel };

// Record a timing event (a recycled one when available) on stream s.
int mark(farms_handle *h, hipStream_t s, hipEvent_t *out) {
    if (!h->ev_free.empty()) {
        *out = h->ev_free.back();
        h->ev_free.pop_back();
    } else {
        HIPCHK(hipEventCreate(out));
    }
    HIPCHK(hipEventRecord(*out, s));
    return FARMS_OK;
}

// Read every pending bracket into h->acc (waits for their end events), then
// the work counters; the events go back to the free list.
// Wall time during which at least one interval runs (intervals as {start, end}).
double union_ms(std::vector<std::pair<double, double>> &iv) {
    std::sort(iv.begin(), iv.end());
    double busy = 0, lo = 0, hi = 0;
    bool open = false;
    for (const auto &v : iv) {
        if (open && v.first <= hi) {
            hi = std::max(hi, v.second);
            continue;
        }
        if (open) busy += hi - lo;
        lo = v.first, hi = v.second, open = true;
    }
    if (open) busy += hi - lo;
    return busy;
}

int harvest(farms_handle *h) {
    std::vector<hipEvent_t> used;
    used.reserve(2 * h->brk.size());
    // the kernel brackets on the device timeline (ms after the first bracket's
    // start, negative if before): their union is the wall time during which a
    // fit (pooling) launch runs, whatever the streams overlap -- the sum of the
    // brackets counts overlapping launches of two fit streams twice
    std::vector<std::pair<double, double>> iv_fit, iv_pool;
    for (const auto &b : h->brk) {
        HIPCHK(hipEventSynchronize(b.b));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, b.a, b.b));
        if (b.kind == kBrFitKernel || b.kind == kBrPoolKernel) {
            float t0 = 0;
            HIPCHK(hipEventElapsedTime(&t0, h->brk.front().a, b.a));
            (b.kind == kBrFitKernel ? iv_fit : iv_pool).emplace_back((double)t0, (double)t0 + (double)ms);
        }
        switch (b.kind) {
        case kBrPrep: h->acc.ms_prep += ms; break;
        case kBrFitSweep: h->acc.ms_fit += ms; break;
        case kBrPoolSweep: h->acc.ms_pool += ms; break;
        case kBrFitKernel: h->acc.ms_fit_kernel += ms; break;
        default: h->acc.ms_pool_kernel += ms; break;
        }
        used.push_back(b.a);
        used.push_back(b.b);
    }
    h->acc.ms_fit_busy += union_ms(iv_fit);
    h->acc.ms_pool_busy += union_ms(iv_pool);
    h->brk.clear();
    std::sort(used.begin(), used.end());
    used.erase(std::unique(used.begin(), used.end()), used.end());
    h->ev_free.insert(h->ev_free.end(), used.begin(), used.end());
    h->acc.ms_total = h->acc.ms_prep + h->acc.ms_pool;
    if (h->counters_dirty) {
        for (hipStream_t s : {h->stream, h->s_chain, h->s_pool, h->s_copy})
            if (s) HIPCHK(hipStreamSynchronize(s));
        unsigned long long cnt[8];
        HIPCHK(hipMemcpy(cnt, h->counters, sizeof(cnt), hipMemcpyDeviceToHost));
        HIPCHK(hipMemset(h->counters, 0, sizeof(cnt)));
        h->acc.n_valid += (int64_t)cnt[0];
        h->acc.sae_cells += (double)cnt[1];
        h->acc.pool_cells += (double)cnt[2];
        h->acc.pool_candidates += (double)cnt[3];
        h->acc.pool_contributors += (double)cnt[4];
        h->acc.n_owned += (int64_t)cnt[5];
        h->acc.pool_scan_over_1k += (int64_t)cnt[6];
        h->acc.pool_scan_max = std::max(h->acc.pool_scan_max, (int64_t)cnt[7]);
        h->counters_dirty = false;
    }
    return FARMS_OK;
}

// Forget the stats (farms_reset): drop the pending brackets, zero the counters.
int clear_stats(farms_handle *h) {
    for (const auto &b : h->brk) {
        h->ev_free.push_back(b.a);
        h->ev_free.push_back(b.b);
    }
    h->brk.clear();
    std::sort(h->ev_free.begin(), h->ev_free.end());
    h->ev_free.erase(std::unique(h->ev_free.begin(), h->ev_free.end()), h->ev_free.end());
    h->acc = farms_stats{};
    h->counters_dirty = false;  // (the device counters: zeroed by reset_surfaces' fill)
    return FARMS_OK;
}

int reset_surfaces(farms_handle *h) {
    int rc = sync_all(h);
    if (rc) return rc;
    // tag 0: never visited, never touched (chunk seqs start at 1)
    // both SAE buffers, each WH cells and a guard head (index WH, never written:
    // the fit reads it for cells outside the stored region); every fill in one
    // launch (k_fill)
    FillTable ft{};
    auto fill = [&](void *ptr, size_t bytes, uint32_t pat) {
        ft.p[ft.n] = ptr;
        ft.words[ft.n] = (int64_t)(bytes / 4);
        ft.pat[ft.n] = pat;
        ++ft.n;
    };
    fill(h->sae_head, 2 * sizeof(SaeHead) * (h->WH + 1), 0u);
    fill(h->sae_tail, 2 * sizeof(SaeTail) * (h->WH + 1), 0u);
    fill(h->ftime, sizeof(int64_t) * h->WH, 0xFFFFFFFFu);  // -1: no valid flow
    fill(h->fsnap, sizeof(FlowCell) * h->WH, 0u);
    for (Work &w : h->ws) {
        fill(w.pcur, sizeof(int32_t) * h->WH, 0u);
        fill(w.pend, sizeof(int32_t) * h->WH, 0xFFFFFFFFu);
        fill(w.cinfo, sizeof(int) * kCiWords, 0u);
    }
    fill(h->counters, sizeof(unsigned long long) * 8, 0u);
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, h->stream, ft);
    HIPCHK(hipStreamSynchronize(h->stream));
    if ((rc = clear_stats(h))) return rc;
    h->seq = 0;
    h->chunk_base = h->super_base = 0;
    h->ph_count = 0;  // fits not pooled are dropped
    h->first_q = -1;
    h->fresh = true;
    return FARMS_OK;
}

template <int K, bool W7>
void launch_pool(const Ctx &c, int c0, int c1, hipStream_t s) {
    const size_t lds = sizeof(uint64_t) * (size_t)(c.pool_bw + c.pool_rs + kPoolValWords);
    hipLaunchKernelGGL((k_pool<K, W7>), dim3(c1 - c0), dim3(64), lds, s, c, c0, c1);
}

typedef void (*pool_launcher)(const Ctx &, int, int, hipStream_t);
template <bool W7>
pool_launcher pool_for_cap(int K) {
    switch (K) {
    case 1: return launch_pool<1, W7>;   case 2: return launch_pool<2, W7>;   case 3: return launch_pool<3, W7>;
    case 4: return launch_pool<4, W7>;   case 5: return launch_pool<5, W7>;   case 6: return launch_pool<6, W7>;
    case 7: return launch_pool<7, W7>;   case 8: return launch_pool<8, W7>;   case 9: return launch_pool<9, W7>;
    case 10: return launch_pool<10, W7>; case 11: return launch_pool<11, W7>; case 12: return launch_pool<12, W7>;
    case 13: return launch_pool<13, W7>; case 14: return launch_pool<14, W7>; case 15: return launch_pool<15, W7>;
    case 16: return launch_pool<16, W7>;
    default: return nullptr;
    }
}
// k_pool's occupancy cap by the fit's weight (see k_pool): 7 waves per SIMD
// beside the quad fits (fs <= 7), 6 beside the wave fits of larger filters.
// (fs 7 wanted 6 while its fit ran on one stream; on two, 7 wins: C4 63.4
// against 64.6 ms, C5 73.5 against 76.4 on a 50M-event share,
// profiles/r04_ab_pool_cap_fs7.log.)  FARMS_POOL_CAP=6|7 overrides (tuning aid).
bool pool_w7(int fr) {
    bool w7 = fr <= 3;
    if (const char *v = getenv("FARMS_POOL_CAP")) w7 = v[0] == '7';
    return w7;
}
pool_launcher pool_for(int K, int fr) {
    return pool_w7(fr) ? pool_for_cap<true>(K) : pool_for_cap<false>(K);
}
// Paired pooling (k_pool2, 2 <= K <= 11): grid = pair slots of chunks [ch0, ch1).
template <int K, bool W7>
void launch_pool2(const Ctx &c, int ch0, int ch1, const int32_t *nv, int4 *ovf, int *ovfn, hipStream_t s) {
    const size_t lds = sizeof(uint64_t) * 2 * (size_t)pair_half_words(pair_bw(c.pool_bw), c.pool_rs);
    hipLaunchKernelGGL((k_pool2<K, W7>), dim3((ch1 - ch0) * (c.C2 >> 1)), dim3(64), lds, s, c, ch0, ch1, nv, ovf,
                       ovfn);
}
// The overflow list of a k_pool2 launch (events past the pair bitmap), pooled
// one event per wave right after it on the pooling stream.  (On the chain
// stream instead, ahead of k_true_polar, its pooling-sized waves waited for
// slots beside the pooling and held the next super-chunk's candidate build:
// C2 2.95 -> 4.8 ms per call, profiles/r06_ab_ovf_stream_c2.log.)
template <int K, bool W7>
void launch_pool_ovf(const Ctx &c, const int4 *ovf, const int *ovfn, hipStream_t s) {
    const size_t lds1 = sizeof(uint64_t) * (size_t)(c.pool_bw + c.pool_rs + kPoolValWords);
    hipLaunchKernelGGL((k_pool_ovf<K, W7>), dim3(kPoolOvfBlocks), dim3(64), lds1, s, c, ovf, ovfn);
}
typedef void (*pair_launcher)(const Ctx &, int, int, const int32_t *, int4 *, int *, hipStream_t);
typedef void (*ovf_launcher)(const Ctx &, const int4 *, const int *, hipStream_t);
template <bool W7>
ovf_launcher ovf_for_cap(int K) {
    switch (K) {
    case 2: return launch_pool_ovf<2, W7>;   case 3: return launch_pool_ovf<3, W7>;   case 4: return launch_pool_ovf<4, W7>;
    case 5: return launch_pool_ovf<5, W7>;   case 6: return launch_pool_ovf<6, W7>;   case 7: return launch_pool_ovf<7, W7>;
    case 8: return launch_pool_ovf<8, W7>;   case 9: return launch_pool_ovf<9, W7>;   case 10: return launch_pool_ovf<10, W7>;
    case 11: return launch_pool_ovf<11, W7>;
    default: return nullptr;
    }
}
template <bool W7>
pair_launcher pair_for_cap(int K) {
    switch (K) {
    case 2: return launch_pool2<2, W7>;   case 3: return launch_pool2<3, W7>;   case 4: return launch_pool2<4, W7>;
    case 5: return launch_pool2<5, W7>;   case 6: return launch_pool2<6, W7>;   case 7: return launch_pool2<7, W7>;
    case 8: return launch_pool2<8, W7>;   case 9: return launch_pool2<9, W7>;   case 10: return launch_pool2<10, W7>;
    case 11: return launch_pool2<11, W7>;
    default: return nullptr;  // one event per wave (k_pool)
    }
}
// Pairs are the default beside the fs <= 5 fits: C3 75.4 -> 73.0 ms per step.
// Beside the fs-7 fit (10.8 KB of LDS per wave, the sweep that paces C4/C5)
// the pairs' 6.4 KB per wave first cost fit waves: C4 54.5 -> 55.8 ms
// (profiles/r05_ab_pool_pairs.log).  With the 4.1-KB pair bitmap and the
// band-contiguous slots they pay at 11 scales (C4 53.1 -> 52.8 ms) and still
// not at 3 (C5 63.2 -> 66.2, profiles/r05_ab_pairs_fs7_final.log): at fs 7
// pairs from 8 scales up.  FARMS_POOL_PAIRS=0|1 overrides (A/B and test aid;
// the same bits).  Pairs need even pooling chunks (the pair slots of a chunk).
pair_launcher pair_for(int K, int fr, int pool_chunk) {
    bool on = fr <= 2 || K >= 8;
    if (const char *v = getenv("FARMS_POOL_PAIRS")) on = v[0] != '0';
    if (!on || (pool_chunk & 1)) return nullptr;
    return pool_w7(fr) ? pair_for_cap<true>(K) : pair_for_cap<false>(K);
}
ovf_launcher ovf_for(int K, int fr) { return pool_w7(fr) ? ovf_for_cap<true>(K) : ovf_for_cap<false>(K); }
// Tuning knobs of the fit (A/B aids; every choice gives the same bits):
// FARMS_FIT_QUAD=0: one thread per event; FARMS_FIT_MODE 0 = re-gather the
// winning window, 1 = union tile with columns per lane (default), 2 = union
// tile with rows per lane.  (Round 4 also measured a wave-wide SAE box in LDS
// and a split of the fit into that box scan plus one lane per event for the
// LU and the ordered sums: C3 / C4 106.7 / 102.4 and 105.4 / 103.4 ms per
// step against 88.9 / 86.9 for mode 1; removed.  DESIGN.md §8.)
bool fit_quad_env() {
    const char *fq = getenv("FARMS_FIT_QUAD");
    return !(fq && fq[0] == '0');
}
// FARMS_ORDER=sort: the work order by the device-wide radix sort even where
// k_chunk_order covers the pooling chunk (A/B and test aid; same bits)
bool order_by_chunk() {
    const char *v = getenv("FARMS_ORDER");
    return !(v && v[0] == 's');
}
// FARMS_CAND=events|chain: force the candidate build (A/B and test aid; every
// choice gives the same bits); default: k_cand for time-local streams.
int cand_force() {
    const char *v = getenv("FARMS_CAND");
    if (!v) return 0;
    return v[0] == 'e' ? 1 : v[0] == 'c' ? 2 : 0;
}
// The fit sweep on one stream or on two (even / odd chunks): two for the
// fit-bound filters (fs 7: C4 73.4 -> 64.8 ms per step), one below, where the
// pooling paces the step and a second fit stream takes its slots (C3 80.0 ->
// 81.6 ms; profiles/r04_ab_fit_streams.log).  FARMS_FIT_STREAMS=1|2 overrides
// (A/B aid, every choice gives the same bits).
int fit_streams_for(int fr) {
    const char *v = getenv("FARMS_FIT_STREAMS");
    if (v && (v[0] == '1' || v[0] == '2')) return v[0] - '0';
    return fr >= 3 ? 2 : 1;
}
int fit_mode_env() {
    const char *fu = getenv("FARMS_FIT_MODE");
    const int m = fu ? atoi(fu) : 1;
    return m >= 0 && m <= 2 ? m : 1;
}

// Fit of chunk [c0, c1); pr.blocks > 0: with the next chunk's prep riding on
// the same launch (quad path only; returns false when it did not take it).
bool launch_fit(const Ctx &c, int fr, int c0, int c1, uint32_t seq, hipStream_t s, bool quad, int mode,
                FitPrep pr) {
    if (quad) {
        const dim3 g(ceil_div(c1 - c0, kFitQS) + pr.blocks), b(64);
#define FARMS_FIT_CASE(FR_)                                                                            \
    if (mode == 2) hipLaunchKernelGGL((k_fit_quad<FR_, 2>), g, b, 0, s, c, c0, c1, seq, pr);          \
    else if (mode == 1) hipLaunchKernelGGL((k_fit_quad<FR_, 1>), g, b, 0, s, c, c0, c1, seq, pr);     \
    else hipLaunchKernelGGL((k_fit_quad<FR_, 0>), g, b, 0, s, c, c0, c1, seq, pr);                    \
    return true;
        switch (fr) {
        case 1: FARMS_FIT_CASE(1)
        case 2: FARMS_FIT_CASE(2)
        case 3: FARMS_FIT_CASE(3)
        default: return false;
        }
#undef FARMS_FIT_CASE
    }
    const dim3 g(ceil_div(c1 - c0, 256)), b(256);
    switch (fr) {
    case 1: hipLaunchKernelGGL(k_fit<1>, g, b, 0, s, c, c0, c1, seq); break;
    case 2: hipLaunchKernelGGL(k_fit<2>, g, b, 0, s, c, c0, c1, seq); break;
    case 3: hipLaunchKernelGGL(k_fit<3>, g, b, 0, s, c, c0, c1, seq); break;
    default: break;  // k_fit_wave
    }
    return false;
}


// FARMS_PLAN_CHECK=1 (test aid): a call with a host-side plan (cand_hint) also
// waits for the device's and fails on a difference.
bool plan_check() {
    const char *v = getenv("FARMS_PLAN_CHECK");
    return v && v[0] == '1';
}

// The candidate plan's reach (k_cand_plan_max / k_cand_plan_back, restated on
// the host): the chunks' min / max stamps tmin / tmax in stream order; for each
// chunk, the distance back to the first earlier chunk whose prefix-maximum
// last stamp lies inside its kill window; the largest such distance.
int host_plan_reach(const std::vector<uint32_t> &tmin, const std::vector<uint32_t> &tmax) {
    const int nch = (int)tmin.size();
    std::vector<uint32_t> pmax(nch);
    uint32_t run = 0;
    for (int i = 0; i < nch; ++i) pmax[i] = run = std::max(run, tmax[i]);
    int reach = 0;
    for (int ch = 0; ch < nch; ++ch) {
        const int64_t lo = (int64_t)tmin[ch] - (int64_t)kKillUs;
        const int a = (int)(std::upper_bound(pmax.begin(), pmax.begin() + ch, lo,
                                             [](int64_t v, uint32_t m) { return (int64_t)m > v; }) -
                            pmax.begin());
        reach = std::max(reach, ch - a);
    }
    return reach;
}

// FARMS_FINISH_LAG (A/B aid): 1 finishes super-chunk S - 1 behind the chain's
// work for S (the round-5 order), 2 (default) S - 2; the ring (3B + 1) holds either.
int finish_lag() {
    const char *v = getenv("FARMS_FINISH_LAG");
    return v && v[0] == '1' ? 1 : 2;
}

int ensure_sync_events(Work &w, size_t count) {
    while (w.sync_ev.size() < count) {
        hipEvent_t ev;
        HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        w.sync_ev.push_back(ev);
    }
    return FARMS_OK;
}

// The whole per-event loop for n device-resident events, with workspace set w.
// on_super (may be null) is called as soon as the work of pooling super-chunk
// S (events [p0, p1)) is enqueued, with the event that marks its records final
// on the device: the host-array path starts the download of those records
// there.  phase 0 runs the whole loop; phase 1 only prep and the local fits
// (then synchronizes), phase 2 only the pooling sweep of the events phase 1
// saw: the x-strip exchange of halo flows (farms_import_flows) goes between
// the two.
// Asynchronous calls (phase 0, `async`; the host-array path's sub-batches)
// return once everything is enqueued: every stream's work of the call is
// ordered before w.done, consecutive calls chain on the streams (F: SAE, C:
// flow snapshots and cursors, P), the candidate ring continues by chunk number,
// and `validated` skips the device-side range check (and its host sync).
typedef std::function<int(int S, int p0, int p1, hipEvent_t done)> super_hook;
// The kernels' view of one call on workspace set w.
Ctx make_ctx(farms_handle *h, Work &w, const int32_t *dx, const int32_t *dy, const uint32_t *dt, const int32_t *dp,
             int n, farms_records *dout, bool async) {
    Ctx c{};
    c.W = h->W; c.H = h->H; c.n = n; c.WH = h->WH; c.WHs = (int64_t)h->W * h->H;
    c.X0 = h->X0; c.XR1 = h->X0 + h->WR; c.own_lo = h->own_lo; c.own_hi = h->own_hi;
    c.fit_lo = h->prm.import_halo ? h->own_lo : h->X0;
    c.fit_hi = h->prm.import_halo ? h->own_hi : h->X0 + h->WR;
    c.fit_all = c.fit_lo <= h->X0 && c.fit_hi >= h->X0 + h->WR;
    c.fr = h->fr; c.min_inl = h->prm.min_inliers; c.J = h->J; c.M = h->M;
    c.invJ = 1.0f / (float)h->J;
    c.kmagic = h->J > 1 ? (uint32_t)(((uint64_t(1) << 32) + (uint64_t)h->J - 1) / (uint64_t)h->J) : 0u;
    c.x = dx; c.y = dy; c.t = dt; c.p = dp;
    c.pix = w.pix; c.skey = w.skey; c.P = w.P; c.link = w.link;
    c.Q = w.Q; c.qe = w.qe; c.fdesc = w.fdesc; c.plane = w.plane;
    c.cells = SaeBuf{h->sae_head, h->sae_tail}; c.PT = w.PT; c.fsnap = h->fsnap; c.ftime = h->ftime;
    c.evf = w.evf; c.valid = w.valid; c.ctmin = w.ctmin; c.ctmax = w.ctmax;
    c.pcur = w.pcur; c.pend = w.pend;
    c.cbk = w.cbk; c.slist = w.slist; c.cinfo = w.cinfo; c.cscr = h->cscr;
    c.bstart = w.bstart; c.nbands = h->nbands; c.bandc = h->bandc; c.band_slots = 0;
    c.s2x = w.s2x; c.s2b = w.s2b;
    c.tshift = h->tile_shift; c.tilesH = (h->H + (1 << h->tile_shift) - 1) >> h->tile_shift;
    c.serial = h->prm.serial != 0;
    c.bw_ring = h->bw_ring; c.nblk = h->nblk; c.cstride = h->cstride;
    c.hdr_ring = h->hdr_ring; c.val_ring = h->val_ring;
    c.nwords = h->nwords; c.NB = h->NB; c.C2 = h->pool_chunk;
    c.ring0 = (int)(h->chunk_base % h->NB);
    const int span = 2 * h->M + 1;  // pooling window rows and columns
    c.pool_bw = (span * span + 63) / 64 + 1;  // flattened window positions (+1: a two-half step reads a word ahead)
    c.pool_rs = span;                     // <= 2 segments per window row, 4 B each
    c.r_true = dout->r_true; c.th_true = dout->theta_true; c.vx = dout->vx; c.vy = dout->vy;
    c.r_local = dout->r_local; c.th_local = dout->theta_local; c.scale = dout->scale;
    c.ox = dout->x; c.oy = dout->y; c.ot = dout->t; c.op = dout->p;
    if (!c.ox || !c.oy || !c.ot || !c.op) c.ox = c.oy = c.ot = c.op = nullptr;
    c.counters = h->counters;
    c.dbg_tc = h->counting ? w.dbg_tc : nullptr;
    (void)async;

    return c;
}

// Before a call writes workspace set w: wait for the set's previous
// asynchronous call, size its dependency events (and the profiling events).
int claim_set(farms_handle *h, Work &w, int n, hipEvent_t *t_start) {
    hipStream_t s = h->stream;
    const int n_fit_chunks = ceil_div(n, h->fit_chunk), n_pool_chunks = ceil_div(n, h->pool_chunk);
    const int n_super = ceil_div(n_pool_chunks, h->pool_batch);
    if (w.busy) {  // the set's previous (asynchronous) call is done with it before anything writes it
        HIPCHK(hipStreamWaitEvent(s, w.done, 0));
        w.busy = false;
    }
    if (t_start) {  // profiled: the prep bracket opens here, after any wait
        int rc = mark(h, s, t_start);
        if (rc) return rc;
    }
    return ensure_sync_events(w, 1 + (size_t)n_fit_chunks + 3 * (size_t)n_super);
}

// The prep of a call on set w (stream F): validate, pixel ids, sort by pixel,
// links, fit descriptors, work order; records w.sync_ev[0].
int enqueue_prep(farms_handle *h, Work &w, const Ctx &c, int n, bool validated, hipEvent_t *t_prep) {
    hipEvent_t t_start = nullptr;
    int rc = claim_set(h, w, n, t_prep ? &t_start : nullptr);
    if (rc) return rc;
    hipStream_t s = h->stream;
    if (h->poison) {  // (test aid, farms_handle::poison) after the set's previous call
        const size_t cap = (size_t)w.cap;
        HIPCHK(hipMemsetAsync(w.qe, kPoisonByte, sizeof(int4) * cap, s));
        HIPCHK(hipMemsetAsync(w.fdesc, kPoisonByte, sizeof(int4) * cap, s));
        HIPCHK(hipMemsetAsync(w.link, kPoisonByte, sizeof(int4) * cap, s));
        HIPCHK(hipMemsetAsync(w.plane, kPoisonByte, sizeof(double2) * cap, s));
        HIPCHK(hipMemsetAsync(w.evf, kPoisonByte, sizeof(FlowCell) * cap, s));
        HIPCHK(hipMemsetAsync(w.valid, kPoisonByte, sizeof(uint8_t) * cap, s));
        HIPCHK(hipMemsetAsync(w.ovf, kPoisonByte, sizeof(int4) * cap, s));
    }
    const int n_pool_chunks = ceil_div(n, h->pool_chunk);
    const uint32_t *dt = c.t;
    hipEvent_t ev_prep = w.sync_ev[0];
    if (!validated) {
        // on the copy stream: not behind F's work.  In device calls that stream
        // also runs the odd fit chunks (fs 7), so the host waits for the
        // previous call's odd fits here: in the x-strip pipeline, where the fit
        // of b + 2 is issued under the fit of b + 1, that is the host's one
        // wait per sub-batch (profiles/r05_strips_async_c4.log; the fits of
        // two-phase calls on stream F alone instead: 99.7 against 77.2 ms)
        // The prep below touches only the workspace set (k_prep clamps a bad
        // event's pixel to 0), so it is enqueued at once and the host waits
        // for the check only before the first fit writes the SAE (check_valid,
        // run_core): the sort and links run under the host's round trip.
        hipStream_t sv = h->s_copy;
        HIPCHK(hipMemsetAsync(h->err, 0, sizeof(int), sv));
        hipLaunchKernelGGL(k_validate, dim3(ceil_div(n, 256)), dim3(256), 0, sv, c.x, c.y, n, c.X0, c.XR1, c.H, h->err);
        HIPCHK(hipMemcpyAsync(h->err_pin + 5, h->err, sizeof(int), hipMemcpyDeviceToHost, sv));
        HIPCHK(hipEventRecord(h->val_ev, sv));
        h->val_pending = true;
    }
    // (k_prep's own flag goes to the second word: the events are in range here)
    hipLaunchKernelGGL(k_prep, dim3(ceil_div(n, 256)), dim3(256), 0, s, c, w.pix, w.iota, w.wkey, h->err + 1,
                       h->pool_chunk, h->tile_bits, h->tile_shift);
    size_t bytes = w.cub_bytes;
    HIPCHK(pixel_sort(w.cub_tmp, bytes, w.pix, w.skey, w.iota, w.P, n, end_bit_for(h->WH), s));
    HIPCHK(hipMemsetAsync(w.pend, 0xFF, sizeof(int32_t) * h->WH, s));  // cells without events in this call
    // serial mode: k_link reads the flow snapshots' stamps, final once the
    // previous call's chain is done
    if (c.serial && h->super_base > 0) HIPCHK(hipStreamWaitEvent(s, h->chain_end, 0));
    hipLaunchKernelGGL(k_link, dim3(ceil_div(n, 256)), dim3(256), 0, s, c, w.link, w.PT, h->prm.serial != 0);
    // the work order, fit descriptors, band starts and chunk spans: one
    // workgroup per pooling chunk when a template covers the chunk size
    // (FARMS_ORDER=sort: the device-wide path, A/B and test aid)
    bool ordered = false;
    if (order_by_chunk()) {
        const dim3 g(n_pool_chunks);
        switch (h->pool_chunk) {
        case 2048: hipLaunchKernelGGL((k_chunk_order<256, 8>), g, dim3(256), 0, s, c, h->tile_bits, w.Q, w.bstart,
                                      w.ctmin, w.ctmax); ordered = true; break;
        case 4096: hipLaunchKernelGGL((k_chunk_order<512, 8>), g, dim3(512), 0, s, c, h->tile_bits, w.Q, w.bstart,
                                      w.ctmin, w.ctmax); ordered = true; break;
        case 8192: hipLaunchKernelGGL((k_chunk_order<1024, 8>), g, dim3(1024), 0, s, c, h->tile_bits, w.Q, w.bstart,
                                      w.ctmin, w.ctmax); ordered = true; break;
        // (16,384-event chunks, fs 7: a 1024 x 16 build -- 123 VGPRs, 70 KB of LDS -- took C4 from
        // 62.3-62.5 to 63.2-64.3 ms per step; those keep the device-wide sort)
        default: break;
        }
    }
    if (!ordered) {
        int cb = 1;
        while ((1 << cb) < n_pool_chunks) ++cb;
        if (cb + h->tile_bits > 32) return fail(FARMS_EINVAL, "too many pooling chunks for one call; raise pool_chunk");
        size_t b2 = w.cub_bytes;
        HIPCHK(hipcub::DeviceRadixSort::SortPairs(w.cub_tmp, b2, w.wkey, w.wkey_sorted, w.iota, w.Q, n, 0,
                                                  h->tile_bits + cb, s));
        hipLaunchKernelGGL(k_fit_desc, dim3(ceil_div(n, 256)), dim3(256), 0, s, c);
        hipLaunchKernelGGL(k_band_starts, dim3(ceil_div(n, 256)), dim3(256), 0, s, c, w.wkey_sorted, h->tile_bits,
                           w.bstart);
        hipLaunchKernelGGL(k_chunk_minmax, dim3(n_pool_chunks), dim3(256), 0, s, dt, n, h->pool_chunk, w.ctmin,
                           w.ctmax);
    }
    if (n_pool_chunks > 0) {  // the candidate build's plan: how far back each chunk's kill window reaches
        hipLaunchKernelGGL(k_cand_plan_max, dim3(1), dim3(1024), 0, s, w.ctmin, w.ctmax, n_pool_chunks, w.cpmax,
                           w.cinfo);
        hipLaunchKernelGGL(k_cand_plan_back, dim3(ceil_div(n_pool_chunks, 256)), dim3(256), 0, s, w.ctmin, w.cpmax,
                           n_pool_chunks, w.cbk, w.cinfo);
        HIPCHK(hipMemcpyAsync(h->plan_pin + (&w - h->ws), w.cinfo + kCiMaxBack, sizeof(int), hipMemcpyDeviceToHost, s));
        HIPCHK(hipEventRecord(w.plan_ev, s));
    }
    HIPCHK(hipEventRecord(ev_prep, s));
    if (t_prep) {
        if ((rc = mark(h, s, t_prep))) return rc;
        h->brk.push_back({t_start, *t_prep, kBrPrep});
    }
    return FARMS_OK;
}

// The records of pooling super-chunk Sg are final only once k_true_polar(Sg)
// has run.  Every consumer of its "pooling done" events takes them as final:
// the host path's downloads (on_super), the call's join, gpool (the chain's
// ring reuse, two super-chunks on) and, recorded after the last of them,
// w.done (the workspace set's reuse).  So k_true_polar(Sg) must run on the
// stream those events are recorded on, before them.  Round 3 moved it to the
// chain stream and left the events on P: the downloads and the join raced it
// and copied (Gx, Gy), and 8 of 48 GPU tests failed (the host-path and
// chunking tests, which compare every record).  The launch leaves a ledger
// entry that the recording checks.
void launch_true_polar(farms_handle *h, const Ctx &c, hipStream_t s, int64_t Sg, int p0, int p1) {
    hipLaunchKernelGGL(k_true_polar, dim3(ceil_div(p1 - p0, 256)), dim3(256), 0, s, c, p0, p1);
    h->polar_stream = s;
    h->polar_super = Sg;
}
int record_pool_done(farms_handle *h, hipStream_t s, int64_t Sg, hipEvent_t ev) {
    if (h->polar_stream != s || h->polar_super != Sg)
        return fail(FARMS_EINTERNAL, "pooling super-chunk " + std::to_string(Sg) +
                                         " marked done before its k_true_polar on the same stream");
    HIPCHK(hipEventRecord(ev, s));
    HIPCHK(hipEventRecord(h->gpool[Sg % 4], s));
    return FARMS_OK;
}

int run_core(farms_handle *h, Work &w, const int32_t *dx, const int32_t *dy, const uint32_t *dt, const int32_t *dp,
             int64_t n64, farms_records *dout, const super_hook *on_super = nullptr, int phase = 0,
             bool async = false, bool validated = false, int cand_hint = -1) {
    const int n = (int)n64;
    hipStream_t s = h->stream;
    h->fresh = false;
    Ctx c = make_ctx(h, w, dx, dy, dt, dp, n, dout, async);

    const bool prof = h->profiling;  // timing brackets, read by farms_get_stats (async calls too)
    hipEvent_t t_prep = nullptr;     // prep done on F: the fit sweep's start
    const int n_fit_chunks = ceil_div(n, h->fit_chunk), n_pool_chunks = ceil_div(n, h->pool_chunk);
    const int B = h->pool_batch;
    const int n_super = ceil_div(n_pool_chunks, B);
    {
        int rc = phase == 2 ? claim_set(h, w, n, nullptr) : enqueue_prep(h, w, c, n, validated, prof ? &t_prep : nullptr);
        if (rc) return rc;
    }
    // sync events: [0] prep done, [1 + f] fit chunk f done, then per super-chunk
    // S: cand[S] (its candidate lists built), pool[S] (its pooling done)
    hipEvent_t ev_prep = w.sync_ev[0];  // (phase 2: w.ready)
    auto ev_fit = [&](int f) { return w.sync_ev[1 + f]; };
    auto ev_cand = [&](int S) { return w.sync_ev[1 + n_fit_chunks + 3 * (size_t)S]; };
    auto ev_pool = [&](int S) { return w.sync_ev[2 + n_fit_chunks + 3 * (size_t)S]; };
    auto super_end = [&](int S) { return (int)std::min<int64_t>((int64_t)(S + 1) * B * h->pool_chunk, n); };
    auto ev_pk = [&](int S) { return w.sync_ev[3 + n_fit_chunks + 3 * (size_t)S]; };  // k_pool(S) done
    // phase 2: prepared by phase 1, its fits and the imported flows in place.
    // When an export / import has already drained stream F past `ready`, the
    // chain stream waits for nothing: a wait on that (completed) event, with
    // the next sub-batch's fits enqueued on F behind it since, held the chain
    // and the pooling until those fits had finished -- the fits and the
    // pooling of the x-strip pipeline then ran in turns instead of together
    // (C4 N=4 middle strip 79.7 ms, rocprofv3 timeline in
    // profiles/r05_strip_trace_c4.txt; host call times in
    // profiles/r05_strip_host_times.log).
    if (phase == 2) ev_prep = w.ready_host ? nullptr : w.ready;
    // ---- the two sweeps, enqueued interleaved so that the GPU starts on the
    // pooling chain as soon as the first fits are done:
    //   stream F: local plane fits, chunk after chunk (k_fit_prep, k_fit,
    //     or k_fit_wave for filters without a compile-time fast path);
    //   stream C: the candidate chain, one k_chain per pooling chunk, each
    //     chunk's records into ring buffer (chunk number) % NB (NB = 3B + 1);
    //   stream P: one k_pool per super-chunk of B pooling chunks.
    // Pooling of a chunk reads only its candidate buffer, the per-event flows
    // and P, so it overlaps the chain of later chunks and the fit sweep.
    // FARMS_SERIALIZE=1 puts everything on one stream (profiling aid: kernel
    // durations without overlap).
    const char *ser = getenv("FARMS_SERIALIZE");
    const bool serial = ser && ser[0] == '1';
    hipStream_t sc = serial ? s : h->s_chain, sp = serial ? s : h->s_pool;
    const int64_t sb0 = h->super_base;
    // (Gx, Gy) -> (RTrue, ThetaTrue) of super-chunk T on the chain stream once
    // its k_pool is done; then its records are final (round 4: k_true_polar
    // off the pooling stream, which paces the step at C3; the chain stream,
    // one super-chunk ahead, has the slack)
    pool_launcher pl = pool_for(h->K, h->fr);
    pair_launcher pl2 = pair_for(h->K, h->fr, h->pool_chunk);
    ovf_launcher plo = pl2 ? ovf_for(h->K, h->fr) : nullptr;
    auto finish_super = [&](int T) -> int {
        const int q0 = T * B * h->pool_chunk, q1 = super_end(T);
        HIPCHK(hipStreamWaitEvent(sc, ev_pk(T), 0));
        launch_true_polar(h, c, sc, sb0 + T, q0, q1);
        if (int rc = record_pool_done(h, sc, sb0 + T, ev_pool(T))) return rc;
        if (on_super) {
            int rc = (*on_super)(T, q0, q1, ev_pool(T));
            if (rc) return rc;
        }
        return FARMS_OK;
    };
    const bool fast_fit = h->fr >= 1 && h->fr <= 3;
    const bool fit_quad = fit_quad_env();
    const int fit_mode = fit_mode_env();
    int fit_launches = 0;
    auto fit_chunk_end = [&](int f) { return (int)std::min<int64_t>((int64_t)(f + 1) * h->fit_chunk, n); };
    // The SAE is double-buffered by chunk parity (buffer f % 2 serves chunk f),
    // so the prep of chunk f+1 rides on the launch of fit f: one launch per fit
    // chunk.  Chunk seqs are base + f + 1.
    const uint32_t seq_base = h->seq;
    h->seq += (uint32_t)n_fit_chunks;
    auto cells_of = [&](int f) {
        const size_t o = (size_t)(f & 1) * (size_t)(h->WH + 1);  // (WH cells and the guard head)
        return SaeBuf{h->sae_head + o, h->sae_tail + o};
    };
    auto fit_start = [&](int f) { return f * h->fit_chunk; };
    auto prep_of = [&](int f) {  // the prep of chunk f (into buffer f % 2); blocks for 64-thread blocks
        FitPrep pr{cells_of(f), fit_start(std::max(f - 2, 0)), fit_start(f), fit_chunk_end(f), seq_base + f + 1, 0};
        pr.blocks = ceil_div(std::max(pr.c1 - pr.c0, pr.c0 - pr.p0), 64);
        return pr;
    };
    // Two fit streams (fit_streams_for): chunk f runs on F (even) or F2 (odd).
    // The fit of chunk f reads SAE buffer f % 2 only, and the prep of chunk f
    // (into that buffer) reads nothing a fit writes (stamps and links), so the
    // even and odd chains are independent: the prep of f + 2 waits only for the
    // fit of f on its own stream, and a fit launch's tail overlaps the next
    // chunk's fit instead of idling its slots.  (One stream: the prep of chunk
    // f + 1 rides on the launch of fit f.)  F2 is the copy stream, idle in a
    // device call after its range check: a fifth stream would share a hardware
    // queue with one of the four (HIP maps streams onto GPU_MAX_HW_QUEUES = 4
    // queues round-robin, and the box's runtime kept 4 whatever the variable
    // said), serializing either the two fit streams or the host path's copies
    // behind F's kernels (C4 73.3 ms; C3 host path 103.8 against 89.3 ms).  So
    // the host path, which keeps the copy stream busy, runs one fit stream.
    const bool two = !serial && !on_super && fit_streams_for(h->fr) == 2 && n_fit_chunks > 1;
    auto fit_stream = [&](int f) { return two && (f & 1) ? h->s_copy : s; };
    auto launch_prep = [&](const FitPrep &pr, hipStream_t st) {
        hipLaunchKernelGGL(k_fit_prep, dim3(pr.blocks), dim3(64), 0, st, c, pr.cells, pr.p0, pr.c0, pr.c1, pr.seq);
    };
    auto enqueue_fit = [&](int f) -> int {  // fit chunk f on stream F (or F2)
        if (h->val_pending) {  // the call's range check (enqueue_prep), before anything writes the SAE
            h->val_pending = false;
            HIPCHK(hipEventSynchronize(h->val_ev));
            if (h->err_pin[5]) return fail(FARMS_EINVAL, "event outside the width x height sensor");
        }
        const int c0 = fit_start(f), c1 = fit_chunk_end(f);
        hipStream_t sf = fit_stream(f);
        if (two && f == 1) HIPCHK(hipStreamWaitEvent(sf, w.sync_ev[0], 0));  // F2 starts behind the call's prep
        if (f == 0 || two) launch_prep(prep_of(f), sf);
        Ctx cf = c;
        cf.cells = cells_of(f);
        FitPrep next{};
        if (!two && f + 1 < n_fit_chunks) next = prep_of(f + 1);
        hipEvent_t k0 = nullptr, k1 = nullptr;
        if (prof && h->fit_events) { int rc = mark(h, sf, &k0); if (rc) return rc; }
        bool merged = false;
        if (fast_fit) {
            merged = launch_fit(cf, h->fr, c0, c1, seq_base + f + 1, sf, fit_quad, fit_mode, next);
        } else {  // no per-thread fast path for this filter: every event wave-cooperative
            hipLaunchKernelGGL(k_fit_wave, dim3(kFitWaveBlocks), dim3(256), 0, sf, cf, seq_base + f + 1, w.Q + c0,
                               c1 - c0);
        }
        if (!merged && next.blocks > 0) launch_prep(next, sf);
        if (k0) {
            int rc = mark(h, sf, &k1);
            if (rc) return rc;
            h->brk.push_back({k0, k1, kBrFitKernel});
        }
        ++fit_launches;
        if (f == n_fit_chunks - 1) {  // the SAE after the call in both buffers (streaming state)
            FitPrep fin{cells_of(f), c0, n, n, 0u, 0};
            fin.blocks = ceil_div(n - c0, 64);
            launch_prep(fin, sf);
            // buffer (f + 1) % 2: its last reader is the fit of chunk f - 1
            if (two) HIPCHK(hipStreamWaitEvent(sf, ev_fit(f - 1), 0));
            fin.cells = cells_of(f + 1);
            fin.p0 = fit_start(std::max(f - 1, 0));
            fin.blocks = ceil_div(n - fin.p0, 64);
            launch_prep(fin, sf);
        }
        HIPCHK(hipEventRecord(ev_fit(f), sf));
        if (f == n_fit_chunks - 1) {
            if (sf != s) HIPCHK(hipStreamWaitEvent(s, ev_fit(f), 0));  // F holds the whole sweep from here on
            if (t_prep && phase == 0) {  // the fit sweep's bracket (phase 1 closes it after k_flow)
                hipEvent_t e2 = nullptr;
                int rc = mark(h, s, &e2);
                if (rc) return rc;
                h->brk.push_back({t_prep, e2, kBrFitSweep});
            }
        }
        return FARMS_OK;
    };
    if (ev_prep) HIPCHK(hipStreamWaitEvent(sc, ev_prep, 0));
    hipEvent_t t_pool0 = nullptr;  // the pooling sweep's start: the chain stream past the prep (phase 2: the fits)
    if (prof && phase != 1) { int rc = mark(h, sc, &t_pool0); if (rc) return rc; }
    // the candidate build of the call (k_cand / k_chain), decided on the host
    // from the plan once the first super-chunk's fits are enqueued: the
    // device's plan (a wait for the prep), or cand_hint, the same plan from the
    // host's copy of the stamps (host_plan_reach: the host-array path, whose
    // sub-batches would otherwise each wait for their prep behind the fits of
    // the one before)
    int use_cand = -1;
    auto decide_cand = [&]() -> int {
        const int force = cand_force();
        if (!h->cand_ok) {
            use_cand = 0;
        } else if (force) {
            use_cand = force == 1;
        } else if (cand_hint >= 0 && !plan_check()) {
            use_cand = cand_hint;
        } else {
            HIPCHK(hipEventSynchronize(w.plan_ev));
            use_cand = h->plan_pin[&w - h->ws] <= kCandMaxBack;
            if (cand_hint >= 0 && cand_hint != use_cand)
                return fail(FARMS_EINTERNAL, "host candidate plan differs from the device's");
        }
        h->cand_last = use_cand;
        c.band_slots = use_cand ? 1 : 0;  // (the pooling launches below take c by value)
        if (use_cand)  // the call-start snapshot list (after the previous call's k_cand_commit on C)
            hipLaunchKernelGGL(k_cand_list, dim3(ceil_div(h->WH, 256)), dim3(256), 0, sc, c, w.slist);
        return FARMS_OK;
    };
    int fit_enqueued = 0;
    if (phase == 1) {  // the whole fit sweep and the local flows, then back to the caller
        while (fit_enqueued < n_fit_chunks) {
            int rc = enqueue_fit(fit_enqueued++);
            if (rc) return rc;
        }
        hipLaunchKernelGGL(k_flow, dim3(ceil_div(n, 256)), dim3(256), 0, s, c, 0, n);
        if (t_prep) {
            hipEvent_t e2 = nullptr;
            int rc = mark(h, s, &e2);
            if (rc) return rc;
            h->brk.push_back({t_prep, e2, kBrFitSweep});
        }
        HIPCHK(hipEventRecord(w.ready, s));
        w.ready_host = false;
        if (!async) HIPCHK(hipStreamSynchronize(s));
        HIPCHK(hipGetLastError());
        h->acc.n_events += n;  // counted here; the pooling call (phase 2) counts its pooling work
        h->acc.fit_launches += fit_launches;
        return FARMS_OK;
    }
    if (phase == 2) fit_enqueued = n_fit_chunks;  // fits done (phase 1)
    const int64_t sb = h->super_base;  // global number of this call's first super-chunk
    const int lag = finish_lag();      // super-chunks between a pooling launch and its k_true_polar
    for (int S = 0; S < n_super; ++S) {
        const int ch0 = S * B, ch1 = std::min(n_pool_chunks, ch0 + B);
        const int64_t Sg = sb + S;
        // keep the fit sweep one super-chunk ahead of the chain
        const int need = std::min(n_fit_chunks, ceil_div(std::min<int64_t>((int64_t)(ch1 + B) * h->pool_chunk, n),
                                                         h->fit_chunk));
        while (fit_enqueued < need) {
            int rc = enqueue_fit(fit_enqueued++);
            if (rc) return rc;
        }
        // ring buffers of super-chunk Sg - 3 (this call's or an earlier one's) are free
        if (Sg >= 3) HIPCHK(hipStreamWaitEvent(sc, h->gpool[(Sg - 3) % 4], 0));
        if (h->poison) {  // (test aid) the buffers the candidate build is about to fill
            for (int ch = ch0; ch < ch1; ++ch) {
                const int64_t buf = (c.ring0 + ch) % h->NB;
                HIPCHK(hipMemsetAsync(h->hdr_ring + buf * h->cstride, kPoisonByte, sizeof(CandHdr) * h->cstride, sc));
                HIPCHK(hipMemsetAsync(h->val_ring + buf * h->cstride, kPoisonByte, sizeof(CandVal) * h->cstride, sc));
                HIPCHK(hipMemsetAsync(h->bw_ring + buf * h->nwords, kPoisonByte, sizeof(BmWord) * h->nwords, sc));
            }
        }
        if (phase == 0) {  // the super-chunk's local flows from its planes (phase 2: done by phase 1)
            const int fl = std::min((int)(((int64_t)ch1 * h->pool_chunk - 1) / h->fit_chunk), n_fit_chunks - 1);
            HIPCHK(hipStreamWaitEvent(sc, ev_fit(fl), 0));
            if (two && fl >= 1) HIPCHK(hipStreamWaitEvent(sc, ev_fit(fl - 1), 0));  // the other fit stream
            const int q0 = ch0 * h->pool_chunk, q1 = super_end(S);
            // one-wave blocks: they take slots as the pooling waves free them
            hipLaunchKernelGGL(k_flow, dim3(ceil_div(q1 - q0, 64)), dim3(64), 0, sc, c, q0, q1);
        }
        if (use_cand < 0) { int rc = decide_cand(); if (rc) return rc; }
        if (use_cand) hipLaunchKernelGGL(k_cand_export, dim3((ch1 - ch0) * h->nbands), dim3(64), 0, sc, c, ch0, ch1);
        for (int a = ch0; a < ch1; a += 64) {  // <= 64 chunks per launch (k_chain: their spans in one VGPR)
            const int b = std::min(a + 64, ch1);
            if (use_cand)
                hipLaunchKernelGGL(k_cand, dim3((b - a) * h->nbands), dim3(64),
                               (sizeof(uint64_t) + sizeof(uint32_t)) * (size_t)ceil_div((int64_t)h->bandc * h->H, 64),
                               sc, c, a, b);
            else
                hipLaunchKernelGGL(k_chain, dim3(h->nblk), dim3(64), 0, sc, c, a, b);
        }
        if (pl2) {  // pooled events compacted per chunk, for the pairs
            hipLaunchKernelGGL(k_pool_compact, dim3(ch1 - ch0), dim3(256), 0, sc, c, ch0, ch1, w.nv, w.ovfn + S);
        } else {
            const int q0 = ch0 * h->pool_chunk, q1 = (int)std::min<int64_t>((int64_t)ch1 * h->pool_chunk, n);
            hipLaunchKernelGGL(k_pool_desc, dim3(ceil_div(q1 - q0, 256)), dim3(256), 0, sc, c, q0, q1);
        }
        HIPCHK(hipEventRecord(ev_cand(S), sc));
        HIPCHK(hipStreamWaitEvent(sp, ev_cand(S), 0));
        const int p0 = ch0 * h->pool_chunk, p1 = (int)std::min<int64_t>((int64_t)ch1 * h->pool_chunk, n);
        hipEvent_t k0 = nullptr, k1 = nullptr;
        if (prof) { int rc = mark(h, sp, &k0); if (rc) return rc; }
        if (pl2) {  // the pairs, then their overflow list (events past the pair bitmap)
            pl2(c, ch0, ch1, w.nv, w.ovf + (int64_t)ch0 * h->pool_chunk, w.ovfn + S, sp);
            plo(c, w.ovf + (int64_t)ch0 * h->pool_chunk, w.ovfn + S, sp);
        }
        else pl(c, p0, p1, sp);
        if (prof) {
            int rc = mark(h, sp, &k1);
            if (rc) return rc;
            h->brk.push_back({k0, k1, kBrPoolKernel});
        }
        HIPCHK(hipEventRecord(ev_pk(S), sp));
        // the records of super-chunk S - 2, on the chain stream behind this
        // one's candidate lists (stream P runs nothing but the pooling): the
        // chain's work for S + 1, queued behind that step, waits only for the
        // pooling of S - 2 and so has the pooling of S - 1 and S to run in.
        // (Finishing S - 1 here, with a ring of 2B + 1, gave it the pooling of S
        // alone, and k_true_polar, slowed beside the pooling, held the chain:
        // C2's pooling stream idled between its launches.)
        if (S >= lag) { int rc = finish_super(S - lag); if (rc) return rc; }
    }
    for (int T = std::max(n_super - lag, 0); T < n_super; ++T) { int rc = finish_super(T); if (rc) return rc; }
    while (fit_enqueued < n_fit_chunks) {
        int rc = enqueue_fit(fit_enqueued++);
        if (rc) return rc;
    }
    h->super_base += n_super;
    h->chunk_base += n_pool_chunks;
    if (n_super > 0) {  // k_cand calls: the snapshots advance to the call's last events
        if (use_cand == 1) hipLaunchKernelGGL(k_cand_commit, dim3(ceil_div(h->WH, 256)), dim3(256), 0, sc, c);
        HIPCHK(hipEventRecord(h->chain_end, sc));
    }
    HIPCHK(hipGetLastError());
    if (phase != 2) {
        h->acc.n_events += n;
        h->acc.fit_launches += fit_launches;
    }
    h->acc.pool_launches += n_super;
    // the pooling sweep's bracket, and the work counters of the call's events
    // (after its last pooling launch, before anything reuses the set)
    if (t_pool0) {
        hipEvent_t e3 = nullptr;
        int rc = mark(h, sp, &e3);
        if (rc) return rc;
        h->brk.push_back({t_pool0, e3, kBrPoolSweep});
    }
    if (h->counting) {
        hipLaunchKernelGGL(k_stats, dim3(1024), dim3(256), 0, sp, c);
        h->counters_dirty = true;
    }
    if (async && n_super > 0) {
        // w.done, on stream P after the last pooling launch (which follows the
        // chain's last step) and F's last work of the call (phase 2 has none):
        // the next call's fits on F do not wait for this call's pooling
        if (phase != 2) {
            HIPCHK(hipEventRecord(w.fend, s));
            HIPCHK(hipStreamWaitEvent(sp, w.fend, 0));
        }
        HIPCHK(hipStreamWaitEvent(sp, h->chain_end, 0));  // k_cand_commit reads the set's links and flows
        HIPCHK(hipEventRecord(w.done, sp));
        w.busy = true;
        return FARMS_OK;
    }
    // join: stream F waits for the last chain step and the last pooling launch
    if (n_super > 0) {
        HIPCHK(hipStreamWaitEvent(s, h->chain_end, 0));
        HIPCHK(hipStreamWaitEvent(s, ev_pool(n_super - 1), 0));
    }
    if (h->counting) {  // k_stats ran on P after the last pooling launch
        hipEvent_t e4 = nullptr;
        int rc = mark(h, sp, &e4);
        if (rc) return rc;
        HIPCHK(hipStreamWaitEvent(s, e4, 0));
        h->ev_free.push_back(e4);
    }
    if (async) {
        HIPCHK(hipEventRecord(w.done, s));
        w.busy = true;
        return FARMS_OK;
    }
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipGetLastError());
    return FARMS_OK;
}

}  // namespace

// ===========================================================================
// C ABI

extern "C" const char *farms_last_error(void) { return g_err.c_str(); }

extern "C" int farms_default_params(farms_params *o) {
    if (!o) return fail(FARMS_EINVAL, "null params");
    std::memset(o, 0, sizeof(*o));
    o->width = 320; o->height = 320; o->filter_size = 3; o->min_inliers = 5;  // main.cpp:21-24
    o->window_jump = 5; o->max_window = 50;                                    // vFlow.cpp:73-74
    return FARMS_OK;
}

extern "C" int farms_create(const farms_params *prm, farms_handle **out) {
    if (!prm || !out) return fail(FARMS_EINVAL, "null argument");
    *out = nullptr;
    if (prm->width <= 0 || prm->height <= 0 || (int64_t)prm->width * prm->height > kMaxSlots)
        return fail(FARMS_EINVAL, "sensor size out of range (at most 2^24 - 256 pixels)");
    if (prm->width > 65535 || prm->height > 65535)  // (the fit's AtA products are 24-bit: coordinates < 2^16)
        return fail(FARMS_EINVAL, "sensor width and height must be below 65536");
    if (prm->window_jump <= 0 || prm->max_window < 0) return fail(FARMS_EINVAL, "bad pooling scales");
    if (prm->region_width < 0 || (prm->region_width > 0 && (prm->region_x0 < 0 || prm->region_x0 + prm->region_width > prm->width)))
        return fail(FARMS_EINVAL, "stored region outside the sensor");
    if (prm->own_x1 < 0 || (prm->own_x1 > 0 && (prm->own_x0 < 0 || prm->own_x0 >= prm->own_x1 || prm->own_x1 > prm->width)))
        return fail(FARMS_EINVAL, "bad owned column range");
    if (prm->own_x1 > 0 && prm->region_width > 0) {
        // the stored region must hold every column the owned events read: the
        // pooling window (M left, M + the W-1 clip's alias columns right,
        // vFlow.cpp:1000/1113) and, for fitted events, the SAE window (2 fRad,
        // vFlow.cpp:870-883) -- of the halo events too unless their flows are
        // imported
        int fs = prm->filter_size;
        if (fs < 5) fs = 3;
        if (!(fs % 2)) fs--;
        const int sae = 2 * (fs / 2), M = std::max(prm->max_window, 0);
        const int alias = std::min(prm->height - 1 + M, prm->width - 1) / prm->height;
        const int left = prm->import_halo ? std::max(M, sae) : M + sae;
        const int right = prm->import_halo ? std::max(M + alias, sae) : M + alias + sae;
        if (prm->region_x0 > std::max(0, prm->own_x0 - left) ||
            prm->region_x0 + prm->region_width < std::min(prm->width, prm->own_x1 + right))
            return fail(FARMS_EINVAL, "stored region does not cover the owned columns' halo");
    }
    const int K = prm->max_window / prm->window_jump + 1;
    // spatialPool has maxWindow slots and is indexed with .at() (vFlow.cpp:966,1025)
    if (K > prm->max_window) return fail(FARMS_EINVAL, "more pooling scales than maxWindow (reference throws)");
    if (K > kMaxScales) return fail(FARMS_EINVAL, "at most 16 pooling scales are supported");
    if (prm->max_window > kPoolMaxM) return fail(FARMS_EINVAL, "maxWindow above 63 is not supported");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(FARMS_ENODEV, "no HIP device");
    if (prm->device < 0 || prm->device >= ndev) return fail(FARMS_ENODEV, "device ordinal out of range");
    HIPCHK(hipSetDevice(prm->device));
    farms_handle *h = new (std::nothrow) farms_handle();
    if (!h) return fail(FARMS_ENOMEM, "host allocation");
    h->prm = *prm;
    int fs = prm->filter_size;  // vFlow.cpp:32-34
    if (fs < 5) fs = 3;
    if (!(fs % 2)) fs--;
    h->fr = fs / 2;
    h->W = prm->width; h->H = prm->height;
    h->X0 = prm->region_width > 0 ? prm->region_x0 : 0;
    h->WR = prm->region_width > 0 ? prm->region_width : prm->width;
    h->own_lo = prm->own_x1 > 0 ? prm->own_x0 : 0;
    h->own_hi = prm->own_x1 > 0 ? prm->own_x1 : prm->width;
    h->WH = (int64_t)h->WR * prm->height;
    h->J = prm->window_jump; h->M = prm->max_window; h->K = K;
    if (h->fr == 3) {  // fs 7 (169-cell fits, fewer valid events): measured best at C4, -10% per step
        // (fit chunks stay at the default: 131,072 won while the fit ran on one
        // stream; on two, 65,536 does -- C4 61.0-61.7 against 63.5-63.7 ms, C5
        // 181.5 against 186.2, 32,768: 64.1 / 188.3; profiles/r04_ab_fit_chunk_fs7.log)
        h->pool_chunk = 2 * kDefaultPoolChunk;
        h->pool_batch = kDefaultPoolBatch / 2;
    }
    {  // smaller sensors pool fewer events per chunk: the default scales with the
       // linear size of the stored region (nearest power of two; 320x320: 2048,
       // measured best; an x-strip of 4 or 8 on 1280x720: 4096, so that its
       // chunks span a time closer to a whole-sensor chunk's)
        const int base = h->pool_chunk;
        const double target = h->pool_chunk * std::sqrt((double)h->WR * h->H / (1280.0 * 720.0));
        while (h->pool_chunk > 1024 && h->pool_chunk > target * std::sqrt(2.0)) h->pool_chunk /= 2;
        // regions that keep the base size (the whole 1280x720 sensor, a half
        // strip of it): 4,096-event chunks, whose candidate lists hold fewer
        // cells too old for most of the chunk's events, in longer super-chunks
        // at fs 5 (round 6 sweep, profiles/r06_ab_pool_chunk_sweep.log: C3
        // 66.0 -> 64.7 ms at 4096 x 192, 65.2 at x 128, 66.1 at x 64; C4 51.8
        // -> 48.2 at 4096 x 64, 49.5-50.0 at 8192 x 64/96/128 and 4096 x 128)
        if (h->pool_chunk == base && prm->pool_chunk <= 0) {  // (an explicit chunk keeps its batch default)
            h->pool_chunk = 4096;
            h->pool_batch = h->fr == 3 ? kDefaultPoolBatch : 3 * kDefaultPoolBatch;
        }
    }
    if (prm->fit_chunk > 0) h->fit_chunk = prm->fit_chunk;
    if (prm->pool_chunk > 0) h->pool_chunk = prm->pool_chunk;
    if (prm->pool_batch > 0) h->pool_batch = prm->pool_batch;
    if (h->pool_chunk > (1 << 24)) {
        delete h;
        return fail(FARMS_EINVAL, "pool_chunk above 2^24");
    }
    h->NB = 3 * h->pool_batch + 1;
    h->nwords = (h->WH + 63) / 64;
    h->nblk = (int)((h->WH + kGroupCells - 1) / kGroupCells);
    h->cstride = (int64_t)h->nblk * kGroupCells;
    // fit chunks are whole pooling chunks (Q is grouped by pooling chunk)
    h->fit_chunk = (int)(((int64_t)h->fit_chunk + h->pool_chunk - 1) / h->pool_chunk * h->pool_chunk);
    {
        // FARMS_TILE_SHIFT (2..5, A/B aid): log2 of the work-order tile's edge
        if (const char *ts = getenv("FARMS_TILE_SHIFT")) h->tile_shift = std::max(2, std::min(atoi(ts), 5));
        if (const char *pz = getenv("FARMS_POISON")) h->poison = pz[0] == '1';
        const int tm = (1 << h->tile_shift) - 1;
        const int64_t tiles = (int64_t)((h->W + tm) >> h->tile_shift) * ((h->H + tm) >> h->tile_shift);
        while ((int64_t(1) << h->tile_bits) < tiles) ++h->tile_bits;
        // k_cand's column bands: whole candidate groups (bandc * H a multiple of
        // 256) and whole work-order tile columns
        const int gq = 256 / std::gcd(h->H, 256), tw = 1 << h->tile_shift;
        h->bandc = gq / std::gcd(gq, tw) * tw;
        h->nbands = (h->WR + h->bandc - 1) / h->bandc;
        h->cand_ok = (int64_t)h->bandc * h->H <= (int64_t)64 * 4096;  // LDS bitmap of a band <= 32 KB
    }
    int rc = FARMS_OK;
    auto bail = [&](int code) { farms_destroy(h); return code; };
    // the fit sweep and the candidate chain are the latency-critical dependency
    // path: high priority; the bulk pooling launches fill the remaining CUs
    // (measured and rejected: a CU mask keeping pooling waves off some CUs of
    // each XCD, other priority assignments: DESIGN.md §8).  The copy stream of
    // farms_process is created with them: the runtime maps streams onto
    // GPU_MAX_HW_QUEUES (4) hardware queues, and a copy stream created later,
    // after another library's stream took a queue, shared F's queue (host path
    // 113 instead of 97 ms at C3).
    int prio_lo = 0, prio_hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
    if (const char *v = getenv("FARMS_STREAM_PRIO"))  // =flat: every stream at the low end (A/B aid)
        if (v[0] == 'f') prio_hi = prio_lo;
    if (hipStreamCreateWithPriority(&h->stream, hipStreamNonBlocking, prio_hi) != hipSuccess ||
        hipStreamCreateWithPriority(&h->s_chain, hipStreamNonBlocking, prio_hi) != hipSuccess ||
        hipStreamCreateWithPriority(&h->s_pool, hipStreamNonBlocking, prio_lo) != hipSuccess ||
        hipStreamCreateWithPriority(&h->s_copy, hipStreamNonBlocking, prio_hi) != hipSuccess)  // (device calls: odd fits)
        return bail(fail(FARMS_EHIP, "hipStreamCreate"));
    {
        std::vector<hipEvent_t *> evs = {&h->gpool[0], &h->gpool[1], &h->gpool[2], &h->gpool[3], &h->chain_end, &h->ex_ev, &h->val_ev};
        for (Work &w : h->ws) {
            evs.push_back(&w.done);
            evs.push_back(&w.ready);
            evs.push_back(&w.fend);
            evs.push_back(&w.plan_ev);
        }
        for (hipEvent_t *ev : evs)
            if (hipEventCreateWithFlags(ev, hipEventDisableTiming) != hipSuccess)
                return bail(fail(FARMS_EHIP, "hipEventCreate"));
    }
    if ((rc = dalloc(&h->sae_head, 2 * (h->WH + 1))) || (rc = dalloc(&h->sae_tail, 2 * (h->WH + 1))) ||
        (rc = dalloc(&h->ftime, h->WH)) ||
        (rc = dalloc(&h->fsnap, h->WH)) ||
        (rc = dalloc(&h->bw_ring, h->nwords * h->NB)) || (rc = dalloc(&h->hdr_ring, h->cstride * h->NB)) ||
        (rc = dalloc(&h->val_ring, h->cstride * h->NB)) || (rc = dalloc(&h->err, 8)) || (rc = dalloc(&h->counters, 8)))
        return bail(rc);
    for (Work &w : h->ws)
        if ((rc = dalloc(&w.pcur, h->WH)) || (rc = dalloc(&w.pend, h->WH)) ||
            (rc = dalloc(&w.slist, h->WH)) || (rc = dalloc(&w.cinfo, kCiWords)))
            return bail(rc);
    if ((rc = dalloc(&h->cscr, (size_t)std::min(h->pool_batch, 64) * h->WH))) return bail(rc);
    if (hipHostMalloc((void **)&h->plan_pin, (3 + 8) * sizeof(int)) != hipSuccess)
        return bail(fail(FARMS_EHIP, "hipHostMalloc"));
    h->err_pin = h->plan_pin + 3;  // (one pinned block: freed with plan_pin)
    std::fill(h->err_pin, h->err_pin + 8, 0);
    if ((rc = reset_surfaces(h))) return bail(rc);
    *out = h;
    return FARMS_OK;
}

extern "C" int farms_destroy(farms_handle *h) {
    if (!h) return FARMS_OK;
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    if (h->s_chain) (void)hipStreamSynchronize(h->s_chain);
    if (h->s_pool) (void)hipStreamSynchronize(h->s_pool);
    if (h->s_copy) (void)hipStreamSynchronize(h->s_copy);
    dfree(h->sae_head); dfree(h->sae_tail); dfree(h->ftime); dfree(h->fsnap);
    for (Work &w : h->ws) {
        free_workspace(w);
        dfree(w.pcur); dfree(w.pend); dfree(w.slist); dfree(w.cinfo);
        for (auto &ev : w.sync_ev) (void)hipEventDestroy(ev);
        if (w.done) (void)hipEventDestroy(w.done);
        if (w.ready) (void)hipEventDestroy(w.ready);
        if (w.fend) (void)hipEventDestroy(w.fend);
        if (w.plan_ev) (void)hipEventDestroy(w.plan_ev);
    }
    for (auto &ev : h->gpool)
        if (ev) (void)hipEventDestroy(ev);
    for (auto &ev : h->up_ev)
        if (ev) (void)hipEventDestroy(ev);
    if (h->chain_end) (void)hipEventDestroy(h->chain_end);
    if (h->ex_ev) (void)hipEventDestroy(h->ex_ev);
    if (h->val_ev) (void)hipEventDestroy(h->val_ev);
    if (h->last_buf) (void)hipFree(h->last_buf);
    dfree(h->bw_ring); dfree(h->cscr);
    dfree(h->hdr_ring); dfree(h->val_ring); dfree(h->err); dfree(h->counters);
    for (auto &b : h->brk) {
        h->ev_free.push_back(b.a);
        h->ev_free.push_back(b.b);
    }
    std::sort(h->ev_free.begin(), h->ev_free.end());
    h->ev_free.erase(std::unique(h->ev_free.begin(), h->ev_free.end()), h->ev_free.end());
    for (auto &ev : h->ev_free) (void)hipEventDestroy(ev);
    for (auto &ev : h->copy_ev) (void)hipEventDestroy(ev);
    for (auto &ev : h->final_ev) (void)hipEventDestroy(ev);
    if (h->s_copy) (void)hipStreamDestroy(h->s_copy);
    if (h->pin_in) (void)hipHostFree(h->pin_in);
    if (h->plan_pin) (void)hipHostFree(h->plan_pin);
    if (h->pin_out) (void)hipHostFree(h->pin_out);
    dfree(h->io_x); dfree(h->io_y); dfree(h->io_t); dfree(h->io_p); dfree(h->io_scale);
    for (auto &d : h->io_rec) dfree(d);
    if (h->s_pool) (void)hipStreamDestroy(h->s_pool);
    if (h->s_chain) (void)hipStreamDestroy(h->s_chain);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return FARMS_OK;
}

extern "C" int farms_reset(farms_handle *h) {
    if (!h) return fail(FARMS_EINVAL, "null handle");
    HIPCHK(hipSetDevice(h->prm.device));
    return reset_surfaces(h);
}

extern "C" int farms_set_profiling(farms_handle *h, int enable) {
    if (!h) return fail(FARMS_EINVAL, "null handle");
    h->profiling = enable != 0;
    h->fit_events = enable != 0 && enable != FARMS_PROF_POOL;
    h->counting = enable != 0 && enable != FARMS_PROF_TIMING && enable != FARMS_PROF_POOL;
    return FARMS_OK;
}

#ifdef FARMS_POOL_STAMPS
// Diagnostic builds only: k_pool's per-phase cycle sums (g_pool_stamps), then cleared.
extern "C" int farms_debug_pool_stamps(unsigned long long *out) {
    HIPCHK(hipDeviceSynchronize());
    std::vector<unsigned long long> rows(8 * kStampRows, 0ull);
    HIPCHK(hipMemcpyFromSymbol(rows.data(), HIP_SYMBOL(g_pool_stamps), sizeof(unsigned long long) * rows.size()));
    for (int i = 0; i < 8; ++i) {
        out[i] = 0;
        for (int r = 0; r < kStampRows; ++r) out[i] += rows[8 * r + i];
    }
    std::fill(rows.begin(), rows.end(), 0ull);
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_pool_stamps), rows.data(), sizeof(unsigned long long) * rows.size()));
    return FARMS_OK;
}
#endif

extern "C" int farms_get_stats(const farms_handle *h, farms_stats *out) {
    if (!h || !out) return fail(FARMS_EINVAL, "null argument");
    farms_handle *m = const_cast<farms_handle *>(h);  // reads the pending brackets (opaque handle)
    HIPCHK(hipSetDevice(h->prm.device));
    int rc = harvest(m);
    if (rc) return rc;
    *out = h->acc;
    return FARMS_OK;
}

extern "C" int farms_num_scales(const farms_handle *h) { return h ? h->K : 0; }

extern "C" int farms_kernel_info(const farms_handle *h, char *buf, int32_t len) {
    if (!h || !buf || len <= 0) return fail(FARMS_EINVAL, "null argument");
    const bool fast = h->fr >= 1 && h->fr <= 3, quad = fit_quad_env();
    const int mode = fit_mode_env();
    const std::string fr = std::to_string(h->fr);
    std::string fit;
    if (!fast) fit = "k_fit_wave";
    else if (!quad) fit = "k_fit<" + fr + ">";
    else fit = "k_fit_quad<" + fr + ">";
    // the candidate build the last pooling call enqueued (decided on the host, per call)
    const std::string cand = h->cand_last < 0 ? "" : h->cand_last ? "k_cand" : "k_chain";
    const std::string pool = pair_for(h->K, h->fr, h->pool_chunk) ? "k_pool2" : "k_pool";
    const std::string js = "{\"fit\": \"" + fit + "\", \"fit_mode\": " + std::to_string(fast && quad ? mode : -1) +
                           ", \"pool\": \"" + pool + "<" + std::to_string(h->K) + ">\", \"pool_cap\": " +
                           (pool_w7(h->fr) ? "7" : "6") + ", \"cand_last\": \"" + cand + "\"}";
    std::snprintf(buf, (size_t)len, "%s", js.c_str());
    return FARMS_OK;
}

extern "C" int farms_get_last_event_time(const farms_handle *h, double *out) {
    if (!h || !out) return fail(FARMS_EINVAL, "null argument");
    HIPCHK(hipSetDevice(h->prm.device));
    double *d = nullptr;
    HIPCHK(hipMalloc((void **)&d, sizeof(double) * h->WH));
    hipLaunchKernelGGL(k_last_time, dim3(ceil_div(h->WH, 256)), dim3(256), 0, h->stream, h->sae_head, h->WH, d);
    for (int64_t q = 0; q < (int64_t)h->W * h->H; ++q) out[q] = 0.0;  // columns outside the region
    hipError_t err = hipMemcpyAsync(out + (int64_t)h->X0 * h->H, d, sizeof(double) * h->WH, hipMemcpyDeviceToHost,
                                    h->stream);
    if (err == hipSuccess) err = hipStreamSynchronize(h->stream);
    (void)hipFree(d);
    // serial mode: the first line stamps lastEventTime without entering the SAE
    // (vFlow.cpp:556); it shows until an event fires at that pixel (which marks
    // the pixel's SAE cell visited)
    if (err == hipSuccess && h->first_q >= 0) {
        SaeHead cell{};
        err = hipMemcpy(&cell, h->sae_head + (h->first_q - (int64_t)h->X0 * h->H), sizeof(cell), hipMemcpyDeviceToHost);
        if (err == hipSuccess && !(cell.w & kHeadVisited)) out[h->first_q] = (double)h->first_t;
    }
    if (err != hipSuccess) return fail(FARMS_EHIP, std::string("farms_get_last_event_time: ") + hipGetErrorString(err));
    return FARMS_OK;
}

extern "C" int farms_last_stamps(farms_handle *h, const int32_t *d_x, const int32_t *d_y, const uint32_t *d_t,
                                 int64_t n, int64_t n_head, int64_t *d_head, int64_t *d_full) {
    if (!h || !d_full || (n_head > 0 && !d_head)) return fail(FARMS_EINVAL, "null argument");
    if (n < 0 || n >= INT_MAX || n_head < 0 || n_head > n) return fail(FARMS_EINVAL, "event count out of range");
    if (n > 0 && (!d_x || !d_y || !d_t)) return fail(FARMS_EINVAL, "null array");
    HIPCHK(hipSetDevice(h->prm.device));
    const int64_t WHs = (int64_t)h->W * h->H;
    hipStream_t s = h->stream;
    const int64_t ntiles = ceil_div(WHs, (int64_t)kLastTile);
    if (ntiles <= kLastMaxTiles) {  // bucketed (no scattered global atomics)
        const int nt = (int)ntiles;
        const size_t cnt_bytes = (sizeof(int) * (3 * (size_t)nt + 1) + 15) & ~(size_t)15;
        const size_t need = cnt_bytes + sizeof(int2) * (size_t)n;
        if (need > h->last_cap) {
            HIPCHK(hipStreamSynchronize(s));
            if (h->last_buf) HIPCHK(hipFree(h->last_buf));
            h->last_buf = nullptr;
            h->last_cap = 0;
            HIPCHK(hipMalloc(&h->last_buf, need));
            h->last_cap = need;
        }
        int *cnt = static_cast<int *>(h->last_buf);  // tcount, tcur, toff (+1), then the buckets
        int2 *bucket = reinterpret_cast<int2 *>(static_cast<char *>(h->last_buf) + cnt_bytes);
        int *tcount = cnt, *tcur = cnt + nt, *toff = cnt + 2 * nt;
        HIPCHK(hipMemsetAsync(tcount, 0, sizeof(int) * nt, s));
        const int nb = (int)ceil_div(n, (int64_t)kLastBlock);
        if (nb > 0)
            hipLaunchKernelGGL(k_last_bucket, dim3(nb), dim3(1024), 0, s, d_x, d_y, (int)n, h->W, h->H, nt, tcount, tcur,
                               bucket, 0);
        hipLaunchKernelGGL(k_last_offsets, dim3(1), dim3(1024), 0, s, tcount, nt, toff, tcur);
        if (nb > 0)
            hipLaunchKernelGGL(k_last_bucket, dim3(nb), dim3(1024), 0, s, d_x, d_y, (int)n, h->W, h->H, nt, tcount, tcur,
                               bucket, 1);
        hipLaunchKernelGGL(k_last_tile, dim3(nt), dim3(256), 0, s, bucket, toff, (int)n_head, d_t, WHs, d_head, d_full);
        HIPCHK(hipStreamSynchronize(s));
        HIPCHK(hipGetLastError());
        return FARMS_OK;
    }
    int32_t *last = nullptr;
    HIPCHK(hipMallocAsync((void **)&last, sizeof(int32_t) * WHs, s));
    HIPCHK(hipMemsetAsync(last, 0xFF, sizeof(int32_t) * WHs, s));  // -1: no event
    if (n_head > 0)
        hipLaunchKernelGGL(k_last_index, dim3(ceil_div(n_head, 256)), dim3(256), 0, s, d_x, d_y, 0, (int)n_head, h->W, h->H, last);
    if (d_head) hipLaunchKernelGGL(k_last_stamp, dim3(ceil_div(WHs, 256)), dim3(256), 0, s, last, d_t, WHs, d_head);
    if (n > n_head)
        hipLaunchKernelGGL(k_last_index, dim3(ceil_div(n - n_head, 256)), dim3(256), 0, s, d_x, d_y, (int)n_head, (int)n,
                           h->W, h->H, last);
    hipLaunchKernelGGL(k_last_stamp, dim3(ceil_div(WHs, 256)), dim3(256), 0, s, last, d_t, WHs, d_full);
    HIPCHK(hipFreeAsync(last, s));
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipGetLastError());
    return FARMS_OK;
}

extern "C" int farms_merge_stamps(farms_handle *h, const int64_t *d_in, int32_t count, int64_t *d_out) {
    if (!h || !d_out || (count > 0 && !d_in) || count < 0) return fail(FARMS_EINVAL, "null argument");
    HIPCHK(hipSetDevice(h->prm.device));
    const int64_t WHs = (int64_t)h->W * h->H;
    hipLaunchKernelGGL(k_merge_stamps, dim3(ceil_div(WHs, 256)), dim3(256), 0, h->stream, d_in, count, WHs, d_out);
    HIPCHK(hipStreamSynchronize(h->stream));
    HIPCHK(hipGetLastError());
    return FARMS_OK;
}

extern "C" int farms_seed_sae(farms_handle *h, const int64_t *d_stamp) {
    if (!h || !d_stamp) return fail(FARMS_EINVAL, "null argument");
    HIPCHK(hipSetDevice(h->prm.device));
    Ctx c{};
    c.W = h->W; c.H = h->H; c.WH = h->WH; c.X0 = h->X0; c.cells = SaeBuf{h->sae_head, h->sae_tail};
    hipLaunchKernelGGL(k_seed_sae, dim3(ceil_div(h->WH, 256)), dim3(256), 0, h->stream, c, d_stamp);
    HIPCHK(hipStreamSynchronize(h->stream));
    HIPCHK(hipGetLastError());
    return FARMS_OK;
}

extern "C" int farms_serial_first(farms_handle *h, int32_t x, int32_t y, uint32_t t_abs) {
    if (!h) return fail(FARMS_EINVAL, "null handle");
    if (!h->prm.serial) return fail(FARMS_EINVAL, "farms_serial_first needs a serial-mode handle");
    if (!h->fresh) return fail(FARMS_EINVAL, "farms_serial_first after events: reset the handle first");
    if (x < h->X0 || x >= h->X0 + h->WR || y < 0 || y >= h->H) return fail(FARMS_EINVAL, "event outside the sensor");
    HIPCHK(hipSetDevice(h->prm.device));
    const int64_t q = (int64_t)(x - h->X0) * h->H + y;
    // lastEventTime[x][y] = t_abs (vFlow.cpp:556): the stamp field of the flow
    // snapshot, whose length stays 0 (the cell has no flow yet)
    HIPCHK(hipMemcpy(reinterpret_cast<uint8_t *>(h->fsnap + q) + offsetof(FlowCell, t), &t_abs, sizeof(uint32_t),
                     hipMemcpyHostToDevice));
    h->first_q = (int64_t)x * h->H + y;
    h->first_t = t_abs;
    return FARMS_OK;
}

namespace {
int check_device_call(farms_handle *h, const int32_t *d_x, const int32_t *d_y, const uint32_t *d_t,
                      const int32_t *d_p, int64_t n, const farms_records *d_out) {
    if (!h || !d_out) return fail(FARMS_EINVAL, "null argument");
    if (n < 0 || n > kMaxCallEvents) return fail(FARMS_EINVAL, "event count out of range (at most 2^29 - 1 per device call)");
    if (n > 0 && (!d_x || !d_y || !d_t || !d_p || !d_out->r_true || !d_out->theta_true || !d_out->vx ||
                  !d_out->vy || !d_out->r_local || !d_out->theta_local || !d_out->scale))
        return fail(FARMS_EINVAL, "null array");
    return FARMS_OK;
}
}  // namespace

// Two-phase calls pipeline: farms_fit_device enqueues its sub-batch's prep and
// fits on the next workspace set and returns; the exports / imports act on the
// oldest fit not yet pooled (h->ph[0], whose pooling comes next: with two fits
// pending that is not the most recent one); farms_pool_device enqueues the
// pooling of the oldest fit not
// yet pooled -- asynchronously when a later fit is pending (its fits and the
// halo exchange then run under this pooling), else it waits for the device.
extern "C" int farms_fit_device(farms_handle *h, const int32_t *d_x, const int32_t *d_y, const uint32_t *d_t,
                                const int32_t *d_p, int64_t n, farms_records *d_out) {
    int rc = check_device_call(h, d_x, d_y, d_t, d_p, n, d_out);
    if (rc) return rc;
    if (h->ph_count >= 2) return fail(FARMS_EINVAL, "two fits are already waiting for farms_pool_device");
    HIPCHK(hipSetDevice(h->prm.device));
    const int set = (int)(h->ph_seq % 3);
    Work &w = h->ws[set];
    if (n > 0) {
        if ((rc = ensure_capacity(h, w, n))) return rc;
        if ((rc = run_core(h, w, d_x, d_y, d_t, d_p, n, d_out, nullptr, 1, /*async=*/true))) return rc;
    }
    h->ph[h->ph_count++] = farms_handle::Phase{d_x, d_y, d_p, d_t, n, *d_out, set};
    ++h->ph_seq;
    return FARMS_OK;
}

extern "C" int farms_pool_device(farms_handle *h) {
    if (!h) return fail(FARMS_EINVAL, "null handle");
    if (h->ph_count == 0) return fail(FARMS_EINVAL, "farms_pool_device without a preceding farms_fit_device");
    HIPCHK(hipSetDevice(h->prm.device));
    const farms_handle::Phase f = h->ph[0];
    h->ph[0] = h->ph[1];
    --h->ph_count;
    const bool ahead = h->ph_count > 0;  // a later fit is pending: stay asynchronous
    int rc = FARMS_OK;
    if (f.n > 0) {
        farms_records out = f.out;
        rc = run_core(h, h->ws[f.set], f.x, f.y, f.t, f.p, f.n, &out, nullptr, 2, /*async=*/true);
    }
    if (!rc && !ahead) rc = sync_all(h);
    return rc;
}

// The exchange acts on the oldest fit not yet pooled (h->ph[0]): the fit
// whose pooling comes next.  (With one fit pending that is also the most recent
// one; the asynchronous order issues the fit of b + 2 before the exchange of
// b + 1, two fits pending.)
namespace {
int exchange_args(farms_handle *h, const void *d_idx, int64_t count, const void *d_flows, const char *what) {
    if (!h || (count > 0 && (!d_idx || !d_flows)) || count < 0 || count >= INT_MAX)
        return fail(FARMS_EINVAL, "bad argument");
    if (h->ph_count == 0) return fail(FARMS_EINVAL, std::string(what) + " outside a fit / pool pair");
    HIPCHK(hipSetDevice(h->prm.device));
    return FARMS_OK;
}
}  // namespace

extern "C" int farms_export_flows_async(farms_handle *h, const int32_t *d_idx, int64_t count, double *d_flows) {
    if (int rc = exchange_args(h, d_idx, count, d_flows, "farms_export_flows")) return rc;
    const farms_handle::Phase &f = h->ph[0];
    // on stream F behind the fit's k_flow: a fit issued after this call runs
    // behind the gather, and farms_export_wait waits for the gather only
    if (count > 0) {
        HIPCHK(hipMemsetAsync(h->err + 2, 0, sizeof(int), h->stream));
        hipLaunchKernelGGL(k_export_flows, dim3(ceil_div(count, 256)), dim3(256), 0, h->stream, h->ws[f.set].evf,
                           d_idx, (int)count, (int)f.n, d_flows, h->err + 2);
        HIPCHK(hipMemcpyAsync(h->err_pin + 2, h->err + 2, sizeof(int), hipMemcpyDeviceToHost, h->stream));
    } else {
        h->err_pin[2] = 0;
    }
    HIPCHK(hipEventRecord(h->ex_ev, h->stream));
    HIPCHK(hipGetLastError());
    h->ex_set = f.set;
    return FARMS_OK;
}

extern "C" int farms_export_wait(farms_handle *h) {
    if (!h) return fail(FARMS_EINVAL, "null handle");
    if (h->ex_set < 0) return FARMS_OK;
    HIPCHK(hipSetDevice(h->prm.device));
    HIPCHK(hipEventSynchronize(h->ex_ev));
    h->ws[h->ex_set].ready_host = true;  // the fits of that set are done (the gather ran behind them on F)
    h->ex_set = -1;
    if (h->err_pin[2]) return fail(FARMS_EINVAL, "farms_export_flows: an index outside the fit's events (slot not written)");
    return FARMS_OK;
}

extern "C" int farms_export_flows(farms_handle *h, const int32_t *d_idx, int64_t count, double *d_flows) {
    int rc = farms_export_flows_async(h, d_idx, count, d_flows);
    if (!rc) rc = farms_export_wait(h);
    return rc;
}

extern "C" int farms_import_flows(farms_handle *h, const int32_t *d_idx, int64_t count, const double *d_flows) {
    if (int rc = exchange_args(h, d_idx, count, d_flows, "farms_import_flows")) return rc;
    const farms_handle::Phase &f = h->ph[0];
    Work &w = h->ws[f.set];
    Ctx c{};
    c.t = f.t; c.evf = w.evf; c.valid = w.valid; c.n = (int)f.n;
    h->err_pin[3] = 0;
    if (count > 0) {
        HIPCHK(hipMemsetAsync(h->err + 3, 0, sizeof(int), h->stream));
        hipLaunchKernelGGL(k_import_flows, dim3(ceil_div(count, 256)), dim3(256), 0, h->stream, c, d_idx, (int)count,
                           d_flows, h->err + 3);
        HIPCHK(hipMemcpyAsync(h->err_pin + 3, h->err + 3, sizeof(int), hipMemcpyDeviceToHost, h->stream));
    }
    HIPCHK(hipEventRecord(w.ready, h->stream));  // the pooling of this fit waits for its imports
    HIPCHK(hipStreamSynchronize(h->stream));
    HIPCHK(hipGetLastError());
    w.ready_host = true;
    if (h->err_pin[3]) return fail(FARMS_EINVAL, "farms_import_flows: an index outside the fit's events (skipped)");
    return FARMS_OK;
}

extern "C" int farms_import_flows_async(farms_handle *h, const int32_t *d_idx, int64_t count, const double *d_flows) {
    if (int rc = exchange_args(h, d_idx, count, d_flows, "farms_import_flows")) return rc;
    const farms_handle::Phase &f = h->ph[0];
    Work &w = h->ws[f.set];
    // on the chain stream, behind the fit (w.ready: its phase-1 end on F, or an
    // earlier import's mark): the pooling of this fit runs on that stream after
    // it, and stream F -- with a later fit already queued -- stays free
    hipStream_t sc = h->s_chain;
    HIPCHK(hipStreamWaitEvent(sc, w.ready, 0));
    Ctx c{};
    c.t = f.t; c.evf = w.evf; c.valid = w.valid; c.n = (int)f.n;
    if (count > 0)  // (out-of-range indices skipped; counted in a word nobody reads: the call does not wait)
        hipLaunchKernelGGL(k_import_flows, dim3(ceil_div(count, 256)), dim3(256), 0, sc, c, d_idx, (int)count, d_flows,
                           h->err + 4);
    HIPCHK(hipEventRecord(w.ready, sc));
    HIPCHK(hipGetLastError());
    w.ready_host = false;  // (the pooling's chain waits w.ready: on its own stream, already in order)
    return FARMS_OK;
}

extern "C" int farms_process_device(farms_handle *h, const int32_t *d_x, const int32_t *d_y,
                                    const uint32_t *d_t, const int32_t *d_p, int64_t n, farms_records *d_out) {
    if (!h || !d_out) return fail(FARMS_EINVAL, "null argument");
    if (h->prm.import_halo) return fail(FARMS_EINVAL, "an import_halo handle runs farms_fit_device / farms_pool_device");
    if (h->ph_count > 0) return fail(FARMS_EINVAL, "a farms_fit_device is waiting for farms_pool_device");
    if (n < 0 || n > kMaxCallEvents) return fail(FARMS_EINVAL, "event count out of range (at most 2^29 - 1 per device call)");
    if (n == 0) return FARMS_OK;
    if (!d_x || !d_y || !d_t || !d_p || !d_out->r_true || !d_out->theta_true || !d_out->vx || !d_out->vy ||
        !d_out->r_local || !d_out->theta_local || !d_out->scale)
        return fail(FARMS_EINVAL, "null array");
    HIPCHK(hipSetDevice(h->prm.device));
    // (Round 4: sub-batches of whole super-chunks on alternating workspace sets,
    // so that the prep of sub-batch b + 1 ran under the pooling of b: C3 79.7 /
    // 80.7 / 82.6 ms per step for 2 / 4 / 8 against 80.0 for one call,
    // profiles/r04_ab_dev_subbatches.log; not kept.)
    int rc = ensure_capacity(h, h->ws[0], n);
    if (rc) return rc;
    return run_core(h, h->ws[0], d_x, d_y, d_t, d_p, n, d_out);
}

namespace {

int host_threads() {
    // FARMS_HOST_THREADS: host threads of the staging copies (default 8)
    const char *v = getenv("FARMS_HOST_THREADS");
    const int t = v ? atoi(v) : 8;
    return std::max(1, std::min(t, 64));
}

int ensure_pinned(farms_handle *h, int64_t n) {
    if (n <= h->pin_cap) return FARMS_OK;
    if (h->pin_in) (void)hipHostFree(h->pin_in);
    if (h->pin_out) (void)hipHostFree(h->pin_out);
    h->pin_in = h->pin_out = nullptr;
    h->pin_cap = 0;
    HIPCHK(hipHostMalloc((void **)&h->pin_in, (size_t)n * 16, hipHostMallocDefault));
    HIPCHK(hipHostMalloc((void **)&h->pin_out, (size_t)n * 52, hipHostMallocDefault));
    h->pin_cap = n;
    return FARMS_OK;
}

int ensure_io(farms_handle *h, int64_t n) {
    if (n <= h->io_cap) return FARMS_OK;
    int rc = sync_all(h);
    if (rc) return rc;
    dfree(h->io_x); dfree(h->io_y); dfree(h->io_t); dfree(h->io_p); dfree(h->io_scale);
    for (auto &d : h->io_rec) dfree(d);
    h->io_cap = 0;
    if ((rc = dalloc(&h->io_x, n)) || (rc = dalloc(&h->io_y, n)) || (rc = dalloc(&h->io_t, n)) ||
        (rc = dalloc(&h->io_p, n)) || (rc = dalloc(&h->io_scale, n)))
        return rc;
    for (auto &d : h->io_rec)
        if ((rc = dalloc(&d, n))) return rc;
    h->io_cap = n;
    return FARMS_OK;
}

// Host memory the DMA engines reach directly (hipHostMalloc'd or registered):
// such arrays skip the pinned staging copy.
bool is_pinned(const void *p) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory: not an error here
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// fn(a, b) over [0, n) split into T slices on host threads (inline when one)
template <class Fn>
void host_parallel(int64_t n, int T, int64_t align, Fn &&fn) {
    // slices of at least 2^16 items, multiples of `align`
    int64_t slice = std::max<int64_t>((n + T - 1) / T, 1 << 16);
    slice = (slice + align - 1) / align * align;
    std::vector<std::thread> th;
    for (int64_t a = 0; a < n; a += slice) {
        const int64_t b = std::min(n, a + slice);
        if (b == n && th.empty()) fn(a, b);
        else th.emplace_back([=, &fn] { fn(a, b); });
    }
    for (auto &w : th) w.join();
}

}  // namespace

// Host arrays in and out (the CLI path, vFlow.cpp:214-416 timed region),
// pipelined in sub-batches of whole pooling super-chunks (about an eighth of
// a long call each; consecutive calls are bitwise one call):
//   upload: sub-batch b's events are range-checked and (pageable arrays)
//     copied into pinned staging by host threads, then DMAed on the copy
//     stream into the call's device copies -- while the GPU still computes
//     sub-batch b - 1 (run_core enqueues asynchronously);
//   compute: run_core on workspace set b % 2, chained on the streams behind
//     b - 1;
//   download: as each pooling super-chunk's records become final on the
//     device (run_core's hook records an event), a host thread waits for it
//     and enqueues the copies of its columns -- straight into the caller's
//     arrays when they are pinned (with the x, y, t, p echo from the device
//     copies), else into pinned staging, moved to the caller's arrays (with
//     the echo) by host threads as each copy lands.
// Only the first sub-batch's upload and the last super-chunk's download are
// not hidden by compute.  An event outside the sensor stops the call with
// FARMS_EINVAL before its sub-batch is enqueued (earlier sub-batches of a long
// call have then been processed: reset the handle to start over).
extern "C" int farms_process(farms_handle *h, const int32_t *x, const int32_t *y, const uint32_t *t,
                             const int32_t *p, int64_t n, farms_records *out) {
    if (!h || !out) return fail(FARMS_EINVAL, "null argument");
    if (h->prm.import_halo) return fail(FARMS_EINVAL, "an import_halo handle runs farms_fit_device / farms_pool_device");
    if (h->ph_count > 0) return fail(FARMS_EINVAL, "a farms_fit_device is waiting for farms_pool_device");
    if (n < 0 || n >= INT_MAX) return fail(FARMS_EINVAL, "event count out of range");
    if (n == 0) return FARMS_OK;
    if (!x || !y || !t || !p || !out->x || !out->y || !out->t || !out->p || !out->r_true || !out->theta_true ||
        !out->vx || !out->vy || !out->r_local || !out->theta_local || !out->scale)
        return fail(FARMS_EINVAL, "null array");
    HIPCHK(hipSetDevice(h->prm.device));
    // sub-batches of whole super-chunks, about n / 8 (at least min_sub super-chunks);
    // profiled or counted calls stay one call (their figures are per call)
    const int64_t super = (int64_t)h->pool_chunk * h->pool_batch;
    int64_t sub = n;
    const char *sbv = getenv("FARMS_SUBBATCHES");  // A/B aid: 1 = one call, k = about n / k per sub-batch
    const int64_t nsub = sbv ? std::max(1, atoi(sbv)) : 8;
    const char *trv = getenv("FARMS_HOST_TRACE");   // 1: host timestamps of the pipeline on stderr
    const bool trace = trv && (trv[0] == '1');
    const auto tr0 = std::chrono::steady_clock::now();
    auto tr = [&](const char *what, int b) {
        if (trace)
            std::fprintf(stderr, "[farms host] %8.3f ms %s %d\n",
                         std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tr0).count(),
                         what, b);
    };
    // a sub-batch holds at least FARMS_SUB_MIN (default 8) super-chunks: each
    // costs a prep on stream F whatever its size (C2, 2M events: 5 sub-batches
    // of at most 4 super-chunks put the device at 4.2 ms against 2.9 ms for
    // one call, the host having enqueued everything by 1.7 ms)
    const char *smv = getenv("FARMS_SUB_MIN");
    const int64_t min_sub = smv ? std::max(1, atoi(smv)) : 8;
    if (!h->profiling && !h->counting && nsub > 1) {
        const int64_t per = std::max<int64_t>(min_sub * super, (n / nsub + super - 1) / super * super);
        if (n > 2 * per) sub = per;
    }
    if (sub > kMaxCallEvents) sub = std::max<int64_t>(kMaxCallEvents / super, 1) * super;  // event ids of a sub-batch: 29 bits
    // Sub-batch bounds.  The first sub-batches grow from two super-chunks by 4x
    // up to `sub`: the call's head (the first sub-batch's range check and
    // upload, not hidden by compute: ~2.5 ms at C3 with n / 8) shrinks, and each
    // later upload still hides under the compute of the one before it (an
    // event uploads ~4.7x faster than it computes at C3).  FARMS_SUB_HEAD=0:
    // equal sub-batches (A/B aid; the records are the same either way).
    std::vector<int64_t> bnd{0};
    {
        const char *shv = getenv("FARMS_SUB_HEAD");
        int64_t size = (shv && shv[0] == '0') ? sub : std::min<int64_t>(2 * super, sub);
        while (bnd.back() < n) {
            bnd.push_back(std::min<int64_t>(n, bnd.back() + size));
            size = std::min<int64_t>(4 * size, sub);
        }
    }
    const int nbat = (int)bnd.size() - 1;
    int rc = FARMS_OK;
    for (int k = 0; k < std::min(nbat, 2) && !rc; ++k) rc = ensure_capacity(h, h->ws[k], sub);  // set b % 2
    if (!rc) rc = ensure_io(h, n);
    if (rc) return rc;
    // per array: pinned host memory is DMAed directly, pageable memory goes
    // through the handle's pinned staging
    const void *uin[4] = {x, y, t, p};
    bool pin_in[4], pin_col[6], pin_echo[4];
    bool all_pinned = true;
    for (int k = 0; k < 4; ++k) all_pinned &= (pin_in[k] = is_pinned(uin[k]));
    double *const ucol[6] = {out->r_true, out->theta_true, out->vx, out->vy, out->r_local, out->theta_local};
    int32_t *const uecho[4] = {out->x, out->y, out->t, out->p};
    for (int k = 0; k < 6; ++k) all_pinned &= (pin_col[k] = is_pinned(ucol[k]));
    // the x/y/t/p echo (vFlow.cpp:370-373) by host copies from the caller's
    // inputs, not by D2H from the device copies: 16 B/event less PCIe traffic
    // under the kernels (round 5, C3: the pinned leg, whose echo was DMAed,
    // ran 89.0 ms against 82.2 for the pageable one, whose echo was copied on
    // the host).  FARMS_ECHO_DMA=1: by D2H (A/B aid).
    const char *edv = getenv("FARMS_ECHO_DMA");
    const bool echo_dma = edv && edv[0] == '1';
    for (int k = 0; k < 4; ++k) all_pinned &= (pin_echo[k] = echo_dma && is_pinned(uecho[k]));
    const bool pin_scale = is_pinned(out->scale);
    all_pinned &= pin_scale;
    if (!all_pinned && (rc = ensure_pinned(h, n))) return rc;

    const int T = host_threads();
    // pinned staging: inputs x | y | t | p, records: six double columns, then scale
    int32_t *stg_in[4];
    for (int k = 0; k < 4; ++k) stg_in[k] = h->pin_in ? reinterpret_cast<int32_t *>(h->pin_in) + (size_t)k * n : nullptr;
    const int32_t *src_in[4];
    for (int k = 0; k < 4; ++k) src_in[k] = pin_in[k] ? static_cast<const int32_t *>(uin[k]) : stg_in[k];
    double *pcol[6];
    for (int k = 0; k < 6; ++k) pcol[k] = h->pin_out ? reinterpret_cast<double *>(h->pin_out) + (size_t)k * n : nullptr;
    int32_t *pscale = h->pin_out ? reinterpret_cast<int32_t *>(reinterpret_cast<double *>(h->pin_out) + 6 * (size_t)n)
                                 : nullptr;
    double *dst_col[6];
    for (int k = 0; k < 6; ++k) dst_col[k] = pin_col[k] ? ucol[k] : pcol[k];
    int32_t *const dst_scale = pin_scale ? out->scale : pscale;
    bool any_host_copy = !pin_scale;  // copy-out threads needed
    for (int k = 0; k < 6; ++k) any_host_copy |= !pin_col[k];
    for (int k = 0; k < 4; ++k) any_host_copy |= !pin_echo[k];

    // one completion event per pooling super-chunk of the call, created before
    // the copy-out threads start: the hook must not grow copy_ev while they read it
    {
        int64_t n_super_all = 0;
        for (int k = 0; k < nbat; ++k) n_super_all += ceil_div(ceil_div(bnd[k + 1] - bnd[k], h->pool_chunk), h->pool_batch);
        while ((int64_t)h->copy_ev.size() < n_super_all) {
            hipEvent_t ev;
            HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            h->copy_ev.push_back(ev);
        }
        while ((int64_t)h->final_ev.size() < n_super_all) {
            hipEvent_t ev;
            HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            h->final_ev.push_back(ev);
        }
        // and one per sub-batch upload: every event exists before a thread is
        // spawned, so an early return here never leaves a joinable thread
        while ((int)h->up_ev.size() < nbat) {
            hipEvent_t ev;
            HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            h->up_ev.push_back(ev);
        }
    }
    struct Ready { int64_t S, p0, p1; };
    std::mutex mu;
    std::condition_variable cv;
    std::vector<Ready> ready;
    size_t taken = 0;
    bool closed = false;
    std::atomic<int> bad{0};
    auto worker = [&]() {  // pageable records: copy-out of landed super-chunks, with the x, y, t, p echo
        for (;;) {
            Ready r;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return taken < ready.size() || closed; });
                if (taken >= ready.size()) return;
                r = ready[taken++];
            }
            if (hipEventSynchronize(h->copy_ev[r.S]) != hipSuccess) { bad = 1; continue; }
            const size_t k = (size_t)(r.p1 - r.p0);
            for (int c = 0; c < 6; ++c)
                if (!pin_col[c]) std::memcpy(ucol[c] + r.p0, pcol[c] + r.p0, 8 * k);
            if (!pin_scale) std::memcpy(out->scale + r.p0, pscale + r.p0, 4 * k);
            // x, y, t, p columns echo the inputs (vFlow.cpp:370-373)
            for (int c = 0; c < 4; ++c)
                if (!pin_echo[c])
                    std::memcpy(uecho[c] + r.p0, static_cast<const int32_t *>(uin[c]) + r.p0, 4 * k);
        }
    };
    std::vector<std::thread> pool;
    if (any_host_copy)
        for (int i = 0; i < T; ++i) pool.emplace_back(worker);
    auto finish = [&](int code) {
        {
            std::lock_guard<std::mutex> lk(mu);
            closed = true;
        }
        cv.notify_all();
        for (auto &w : pool) w.join();
        int rs = sync_all(h);
        return code ? code : rs;
    };
    int64_t S_all = 0;  // super-chunks of the call so far
    // Record downloads: a host thread enqueues each super-chunk's copies on the
    // copy stream once its records are final (their event has completed), so
    // the copy queue never holds a wait on the pooling.  Measured (C3, pinned,
    // FARMS_HOST_TRACE=1): with the waits enqueued in the copy queue the copies
    // fell 47-95 ms behind the pooling (more the earlier they were enqueued),
    // although the host enqueued everything within 10 ms; enqueued only when
    // ready they finish within 1 ms of the last pooling launch.
    struct Download { int64_t S, a0; int p0, p1; hipEvent_t done; };
    // the copies of the records [g0, g1) of the call (super-chunks S0..S1 - 1,
    // whose records are final), each super-chunk's completion event after them
    auto enqueue_download = [&](int64_t S0, int64_t S1, int64_t g0, int64_t g1) -> int {
        hipStream_t sd = h->s_copy;
        const size_t k = (size_t)(g1 - g0);
        for (int c = 0; c < 6; ++c)
            HIPCHK(hipMemcpyAsync(dst_col[c] + g0, h->io_rec[c] + g0, 8 * k, hipMemcpyDeviceToHost, sd));
        HIPCHK(hipMemcpyAsync(dst_scale + g0, h->io_scale + g0, 4 * k, hipMemcpyDeviceToHost, sd));
        // the x, y, t, p echo (vFlow.cpp:370-373) of pinned columns from the device copies
        int32_t *const io_in[4] = {h->io_x, h->io_y, h->io_t, h->io_p};
        for (int c = 0; c < 4; ++c)
            if (pin_echo[c]) HIPCHK(hipMemcpyAsync(uecho[c] + g0, io_in[c] + g0, 4 * k, hipMemcpyDeviceToHost, sd));
        for (int64_t S = S0; S < S1; ++S) HIPCHK(hipEventRecord(h->copy_ev[S], sd));
        if (any_host_copy) {
            {
                std::lock_guard<std::mutex> lk(mu);
                ready.push_back(Ready{S1 - 1, g0, g1});
            }
            cv.notify_one();
        }
        return FARMS_OK;
    };
    std::mutex dmu;
    std::condition_variable dcv;
    std::deque<Download> dq;
    bool dclosed = false;
    std::atomic<int> dl_rc{0};
    // The download thread: waits for the oldest pending super-chunk's records,
    // then takes with it the following ones already final (their events
    // complete), so that when the copies lag the compute they go out as one
    // copy per column over several super-chunks: each copy costs ~10 us of
    // DMA set-up besides its bytes (C2: 1-MB copies of 25 us, one every 35 us;
    // the last records landed 1.4 ms after the last pooling launch).
    std::thread dlt([&]() {
        if (hipSetDevice(h->prm.device) != hipSuccess) dl_rc = FARMS_EHIP;
        for (;;) {
            Download q;
            {
                std::unique_lock<std::mutex> lk(dmu);
                dcv.wait(lk, [&] { return !dq.empty() || dclosed; });
                if (dq.empty()) return;
                q = dq.front();
                dq.pop_front();
            }
            if (dl_rc) continue;  // a failed download: drain the queue, the call reports it
            if (hipEventSynchronize(q.done) != hipSuccess) { dl_rc = FARMS_EHIP; continue; }
            int64_t S1 = q.S + 1, g1 = q.a0 + q.p1;
            for (;;) {  // the next ones, while contiguous and final
                std::lock_guard<std::mutex> lk(dmu);
                if (dq.empty()) break;
                const Download &r = dq.front();
                if (r.S != S1 || r.a0 + r.p0 != g1 || hipEventQuery(r.done) != hipSuccess) break;
                S1 = r.S + 1;
                g1 = r.a0 + r.p1;
                dq.pop_front();
            }
            if (int r = enqueue_download(q.S, S1, q.a0 + q.p0, g1)) dl_rc = r;
        }
    });
    auto close_downloads = [&]() {
        {
            std::lock_guard<std::mutex> lk(dmu);
            dclosed = true;
        }
        dcv.notify_all();
        dlt.join();
    };
    // asynchronous sub-batches unless the call is profiled (timing and counters
    // are read back per call)
    const bool async = !h->profiling && !h->counting;
    // range check (vFlow.cpp:264 indexes the surfaces unchecked), staging and
    // upload of sub-batch b into the call's device copies (nothing to wait for)
    // and the sub-batch's candidate plan from the stamps (its pooling chunks
    // start at the sub-batch's start: bounds are whole super-chunks)
    std::vector<int> hint(nbat, -1);
    auto upload = [&](int b) -> int {
        const int64_t a0 = bnd[b], m = bnd[b + 1] - a0;
        const int C2 = h->pool_chunk;
        const int nch = (int)ceil_div(m, (int64_t)C2);
        std::vector<uint32_t> tmin(nch, 0xFFFFFFFFu), tmax(nch, 0u);
        std::atomic<int> oor{0};
        host_parallel(m, T, C2, [&](int64_t i0, int64_t i1) {
            const int64_t e0 = a0 + i0, k = i1 - i0;
            const int xlo = h->X0, xhi = h->X0 + h->WR, H = h->H;
            int o = 0;
            for (int64_t e = e0; e < e0 + k; ++e) o |= (x[e] < xlo) | (x[e] >= xhi) | (y[e] < 0) | (y[e] >= H);
            if (o) oor = 1;
            for (int64_t c0 = i0; c0 < i1; c0 += C2) {  // (slices are whole chunks)
                const uint32_t *tc = t + a0 + c0;
                const int64_t kc = std::min<int64_t>(C2, i1 - c0);
                uint32_t lo = 0xFFFFFFFFu, hi = 0;
                for (int64_t i = 0; i < kc; ++i) { lo = std::min(lo, tc[i]); hi = std::max(hi, tc[i]); }
                tmin[c0 / C2] = lo;
                tmax[c0 / C2] = hi;
            }
            for (int c = 0; c < 4; ++c)
                if (!pin_in[c]) std::memcpy(stg_in[c] + e0, static_cast<const int32_t *>(uin[c]) + e0, 4 * k);
        });
        tr("staged", b);
        if (oor) return fail(FARMS_EINVAL, "event outside the width x height sensor");
        hint[b] = host_plan_reach(tmin, tmax) <= kCandMaxBack ? 1 : 0;
        hipStream_t su = h->s_copy;
        int32_t *const io_in[4] = {h->io_x, h->io_y, h->io_t, h->io_p};
        for (int c = 0; c < 4; ++c)
            if (hipMemcpyAsync(io_in[c] + a0, src_in[c] + a0, 4 * m, hipMemcpyHostToDevice, su) != hipSuccess)
                return fail(FARMS_EHIP, "farms_process: host-to-device copy");
        HIPCHK(hipEventRecord(h->up_ev[b], su));
        tr("uploaded", b);
        return FARMS_OK;
    };
    auto records_of = [&](int64_t a0) {
        farms_records d{};
        d.r_true = h->io_rec[0] + a0; d.theta_true = h->io_rec[1] + a0; d.vx = h->io_rec[2] + a0;
        d.vy = h->io_rec[3] + a0; d.r_local = h->io_rec[4] + a0; d.theta_local = h->io_rec[5] + a0;
        d.scale = h->io_scale + a0;
        return d;
    };
    // The staging thread: range check, chunk stamp ranges (the sub-batch's
    // candidate plan) and upload of each sub-batch, at most `ahead` sub-batches
    // before the compute the main thread enqueues, so that the host's two
    // chores overlap (C2: ~0.3 ms of staging and ~0.4 ms of enqueue per
    // sub-batch, one after the other, were the host path's pace).  The upload
    // of b + 1 goes out before b's compute is enqueued (and before b's
    // downloads, which share the copy stream).  (Pinned inputs uploaded all up
    // front: 1.5 ms slower at C3, the burst of uploads slows the first
    // sub-batches' kernels more.)  FARMS_UPLOAD_AHEAD=0: each sub-batch staged
    // only once the main thread reaches it (A/B aid).
    const char *uav = getenv("FARMS_UPLOAD_AHEAD");
    const int ahead = (uav && uav[0] == '0') ? 0 : 1;
    std::mutex smu;
    std::condition_variable scv;
    int allowed = 0, ok_count = 0, fail_at = -1, st_rc = FARMS_OK;
    bool st_stop = false;
    std::string st_err;
    std::thread stager([&]() {
        int r = hipSetDevice(h->prm.device) == hipSuccess ? FARMS_OK : fail(FARMS_EHIP, "farms_process: staging thread");
        for (int b = 0; b < nbat; ++b) {
            {
                std::unique_lock<std::mutex> lk(smu);
                scv.wait(lk, [&] { return b < allowed || st_stop; });
                if (st_stop) return;
            }
            if (r == FARMS_OK) r = upload(b);
            {
                std::lock_guard<std::mutex> lk(smu);
                if (r) { fail_at = b; st_rc = r; st_err = g_err; }
                else ok_count = b + 1;
            }
            scv.notify_all();
            if (r) return;
        }
    });
    auto stop_stager = [&]() {
        {
            std::lock_guard<std::mutex> lk(smu);
            st_stop = true;
        }
        scv.notify_all();
        stager.join();
    };
    for (int b = 0; b < nbat && !rc; ++b) {
        const int64_t a0 = bnd[b], m = bnd[b + 1] - a0;
        Work &w = h->ws[b & 1];
        {
            std::unique_lock<std::mutex> lk(smu);
            allowed = std::max(allowed, std::min(b + 1 + ahead, nbat));
            scv.notify_all();
            scv.wait(lk, [&] { return ok_count > b || fail_at >= 0; });
            if (ok_count <= b) {  // this sub-batch's staging failed (out-of-range event, copy)
                rc = fail(st_rc, st_err);
                break;
            }
        }
        int32_t *const dev_in[4] = {h->io_x + a0, h->io_y + a0, h->io_t + a0, h->io_p + a0};
        if (hipStreamWaitEvent(h->stream, h->up_ev[b], 0) != hipSuccess) {
            rc = fail(FARMS_EHIP, "farms_process: upload wait");
            break;
        }
        // ---- compute, with the record downloads hooked onto each super-chunk
        farms_records d = records_of(a0);
        super_hook hook = [&](int, int p0, int p1, hipEvent_t) -> int {
            // an event of the call's own (the set's pooling events are recorded again by later sub-batches)
            if ((int64_t)h->final_ev.size() <= S_all || (int64_t)h->copy_ev.size() <= S_all)
                return fail(FARMS_EHIP, "farms_process: super-chunk count");
            HIPCHK(hipEventRecord(h->final_ev[S_all], h->polar_stream));  // where its k_true_polar ran
            {
                std::lock_guard<std::mutex> lk(dmu);
                dq.push_back(Download{S_all, a0, p0, p1, h->final_ev[S_all]});
            }
            ++S_all;
            dcv.notify_one();
            return FARMS_OK;
        };
        rc = run_core(h, w, dev_in[0], dev_in[1], reinterpret_cast<const uint32_t *>(dev_in[2]), dev_in[3], m, &d,
                      &hook, 0, async, /*validated=*/true, hint[b]);
        if (rc) break;
        tr("enqueued", b);
    }
    stop_stager();
    if (trace) {  // when the device finished each stream's work
        (void)hipStreamSynchronize(h->stream); tr("F done", nbat);
        (void)hipStreamSynchronize(h->s_pool); tr("P done", nbat);
    }
    close_downloads();
    if (!rc && dl_rc) rc = fail(dl_rc, "farms_process: record download");
    if (trace) { (void)hipStreamSynchronize(h->s_copy); tr("D2H done", nbat); }
    rc = finish(rc);
    tr("copy-out done", nbat);
    if (rc) return rc;
    if (bad) return fail(FARMS_EHIP, "farms_process: device-to-host copy");
    return FARMS_OK;
}

extern "C" int farms_host_alloc(int64_t bytes, void **out) {
    if (!out || bytes < 0) return fail(FARMS_EINVAL, "bad argument");
    *out = nullptr;
    HIPCHK(hipHostMalloc(out, (size_t)(bytes > 0 ? bytes : 1), hipHostMallocDefault));
    return FARMS_OK;
}

extern "C" int farms_host_free(void *p) {
    if (p) HIPCHK(hipHostFree(p));
    return FARMS_OK;
}
