// farms_synth.cpp — seeded "moving bars" event-stream generator.
//
// Workload tool for tests and bench.py; not part of the accelerated path.  The
// reference ships no data, so the configurations of BASELINE.json
// are synthesised here from documented seeds.
//
// PRNG: SplitMix64 (Steele, Lea, Flood 2014):
//   s += 0x9E3779B97F4A7C15; z = s; z = (z ^ z>>30) * 0xBF58476D1CE4E5B9;
//   z = (z ^ z>>27) * 0x94D049BB133111EB; return z ^ z>>31;
// uniform double = (z >> 11) * 2^-53.  The bars' parameters come from one
// SplitMix64 sequence seeded with `seed`.  Every per-event draw is counter-based
// instead -- the SplitMix64 output function of a hash of the event's identity
// (time step, bar, pixel, edge crossing; noise event number) -- so any block of
// time steps can be generated on its own: blocks run on parallel threads, and a
// rank's share [e0, e1) of a long stream is produced without materialising the
// rest (two passes: per-microsecond counts, then the keys of the window).
//
// Geometry: pixel (px, py) has its centre at (px, py).  A bar is the rectangle
// |(q-c).u| <= L/2, |(q-c).m| <= w/2 with u the long axis and m its normal.  The
// centre moves with constant velocity inside each 100 us step and reflects off
// the sensor border between steps.  For every edge of the rectangle the pixels
// of its swept parallelogram are visited by scanline and the exact entry (ON,
// p=+1) / exit (OFF, p=-1) instant of each pixel centre is solved from the two
// slab intervals; an event is emitted by the edge that binds it, so corners are
// not duplicated.  The signal is simulated step by step until it holds
// n_signal + n_signal/64 + 1024 events (a margin for the tail cut), noise is
// spread uniformly over the simulated span, and the stream is the first
// n_events events in (t, x, y, p) order.
#include "../../include/farms_synth.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

namespace {

struct SplitMix64 {
    uint64_t s;
    explicit SplitMix64(uint64_t seed) : s(seed) {}
    uint64_t next() {
        s += 0x9E3779B97F4A7C15ull;
        uint64_t z = s;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    double uniform() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
    double uniform(double a, double b) { return a + (b - a) * uniform(); }
};

// SplitMix64's output function: the counter-based draw of a hashed identity.
inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

constexpr double kPi = 3.14159265358979323846;
constexpr uint32_t kStepUs = 100;  // motion is linear within a step
constexpr double kStepS = kStepUs * 1e-6;
constexpr int kBlockSteps = 64;    // time steps per generation block (one thread's unit)

struct Bar {
    double cx, cy, vx, vy;  // centre (px) and velocity (px/s)
    double ux, uy, mx, my;  // long axis u, normal m
    double half_len, half_thick;
};

struct V2 { double x, y; };

// Key layout: t (32) | x (16) | y (15) | polarity bit (1) -> sort order (t, x, y, p).
inline uint64_t make_key(uint32_t t, int x, int y, int p) {
    return ((uint64_t)t << 32) | ((uint64_t)(uint32_t)x << 16) | ((uint64_t)(uint32_t)y << 1) |
           (uint64_t)(p > 0 ? 1 : 0);
}
inline int key_x(uint64_t k) { return (int)((k >> 16) & 0xFFFF); }

void radix_sort_u64(std::vector<uint64_t> &a) {
    std::vector<uint64_t> tmp(a.size());
    std::vector<size_t> count(65536);
    for (int pass = 0; pass < 4; ++pass) {
        const int sh = pass * 16;
        std::fill(count.begin(), count.end(), 0);
        for (uint64_t k : a) count[(k >> sh) & 0xFFFF]++;
        size_t sum = 0;
        for (size_t &c : count) { size_t v = c; c = sum; sum += v; }
        for (uint64_t k : a) tmp[count[(k >> sh) & 0xFFFF]++] = k;
        a.swap(tmp);
    }
}

// Interval of tau where |a0 - v*tau| <= h (closed), on the whole real line.
// Returns false when empty.  side_lo/side_hi: which boundary (+h or -h) is hit
// at lo / hi.
inline bool slab(double a0, double v, double h, double &lo, double &hi, int &side_lo, int &side_hi) {
    if (std::fabs(v) < 1e-12) {
        if (std::fabs(a0) <= h) { lo = -INFINITY; hi = INFINITY; side_lo = side_hi = 0; return true; }
        return false;
    }
    double t_plus = (a0 - h) / v;   // a(t) = +h
    double t_minus = (a0 + h) / v;  // a(t) = -h
    if (t_plus < t_minus) { lo = t_plus; hi = t_minus; side_lo = +1; side_hi = -1; }
    else { lo = t_minus; hi = t_plus; side_lo = -1; side_hi = +1; }
    return true;
}

// The events of bar `bi` during time step `step`: sink(t_off, px, py, p) with
// t_off the stamp minus t0 (us).  Jitter U{0..J}: a counter-based draw from
// (seed, step, bar, pixel, entry/exit).
template <class Sink>
void emit_bar_step(const Bar &b, int bi, uint32_t step, int W, int H, int jitter, uint64_t seed, Sink &&sink) {
    const double vu = b.vx * b.ux + b.vy * b.uy;
    const double vm = b.vx * b.mx + b.vy * b.my;
    const V2 dv{b.vx * kStepS, b.vy * kStepS};
    const uint64_t hstep = mix64(seed ^ (((uint64_t)step << 16) | (uint64_t)bi));
    // edges: (slab 0 = u, slab 1 = m) x (side +1, -1)
    for (int slab_id = 0; slab_id < 2; ++slab_id) {
        for (int side = +1; side >= -1; side -= 2) {
            V2 a, c;  // edge endpoints
            if (slab_id == 0) {
                double ox = b.cx + side * b.half_len * b.ux, oy = b.cy + side * b.half_len * b.uy;
                a = {ox - b.half_thick * b.mx, oy - b.half_thick * b.my};
                c = {ox + b.half_thick * b.mx, oy + b.half_thick * b.my};
            } else {
                double ox = b.cx + side * b.half_thick * b.mx, oy = b.cy + side * b.half_thick * b.my;
                a = {ox - b.half_len * b.ux, oy - b.half_len * b.uy};
                c = {ox + b.half_len * b.ux, oy + b.half_len * b.uy};
            }
            V2 poly[4] = {a, c, {c.x + dv.x, c.y + dv.y}, {a.x + dv.x, a.y + dv.y}};
            double xmin = poly[0].x, xmax = poly[0].x;
            for (auto &q : poly) { xmin = std::min(xmin, q.x); xmax = std::max(xmax, q.x); }
            int px0 = std::max(0, (int)std::ceil(xmin - 1e-9));
            int px1 = std::min(W - 1, (int)std::floor(xmax + 1e-9));
            for (int px = px0; px <= px1; ++px) {
                double ylo = INFINITY, yhi = -INFINITY;
                for (int k = 0; k < 4; ++k) {
                    const V2 &p0 = poly[k], &p1 = poly[(k + 1) & 3];
                    double x0 = std::min(p0.x, p1.x), x1 = std::max(p0.x, p1.x);
                    if (px < x0 - 1e-9 || px > x1 + 1e-9) continue;
                    if (std::fabs(p1.x - p0.x) < 1e-12) {
                        ylo = std::min(ylo, std::min(p0.y, p1.y));
                        yhi = std::max(yhi, std::max(p0.y, p1.y));
                    } else {
                        double s = (px - p0.x) / (p1.x - p0.x);
                        s = std::min(1.0, std::max(0.0, s));
                        double yy = p0.y + s * (p1.y - p0.y);
                        ylo = std::min(ylo, yy);
                        yhi = std::max(yhi, yy);
                    }
                }
                if (!(ylo <= yhi)) continue;
                int py0 = std::max(0, (int)std::ceil(ylo - 1e-9));
                int py1 = std::min(H - 1, (int)std::floor(yhi + 1e-9));
                for (int py = py0; py <= py1; ++py) {
                    const double qx = px - b.cx, qy = py - b.cy;
                    double lo_u, hi_u, lo_m, hi_m;
                    int slo_u, shi_u, slo_m, shi_m;
                    if (!slab(qx * b.ux + qy * b.uy, vu, b.half_len, lo_u, hi_u, slo_u, shi_u)) continue;
                    if (!slab(qx * b.mx + qy * b.my, vm, b.half_thick, lo_m, hi_m, slo_m, shi_m)) continue;
                    const double lo = std::max(lo_u, lo_m), hi = std::min(hi_u, hi_m);
                    if (!(lo < hi)) continue;
                    const int bind_lo = lo_u > lo_m ? 0 : 1, bind_hi = hi_u < hi_m ? 0 : 1;
                    const int side_lo = bind_lo == 0 ? slo_u : slo_m, side_hi = bind_hi == 0 ? shi_u : shi_m;
                    for (int which = 0; which < 2; ++which) {
                        const double tau = which == 0 ? lo : hi;
                        if (!(tau >= 0.0 && tau < kStepS)) continue;
                        if ((which == 0 ? bind_lo : bind_hi) != slab_id) continue;
                        if ((which == 0 ? side_lo : side_hi) != side) continue;
                        const uint64_t h = mix64(hstep ^ (((uint64_t)px << 17) | ((uint64_t)py << 1) | (uint64_t)which));
                        const uint32_t tt = step * kStepUs + (uint32_t)std::floor(tau * 1e6) +
                                            (uint32_t)(h % ((uint64_t)jitter + 1));
                        sink(tt, px, py, which == 0 ? +1 : -1);
                    }
                }
            }
        }
    }
}

void advance(std::vector<Bar> &bars, int W, int H) {
    for (Bar &b : bars) {
        b.cx += b.vx * kStepS;
        b.cy += b.vy * kStepS;
        if (b.cx < 0) { b.cx = -b.cx; b.vx = -b.vx; }
        if (b.cx > W - 1) { b.cx = 2.0 * (W - 1) - b.cx; b.vx = -b.vx; }
        if (b.cy < 0) { b.cy = -b.cy; b.vy = -b.vy; }
        if (b.cy > H - 1) { b.cy = 2.0 * (H - 1) - b.cy; b.vy = -b.vy; }
    }
}

int n_threads() {
    // OMP_NUM_THREADS (16 on the GPU boxes, whose nproc shows the whole host) or
    // the hardware count, at most 32
    const char *v = std::getenv("FARMS_SYNTH_THREADS");
    if (!v) v = std::getenv("OMP_NUM_THREADS");
    int t = v ? std::atoi(v) : (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(t, 32));
}

// fn(i) for i in [0, n) on the worker threads
template <class Fn>
void parallel_for(int64_t n, Fn &&fn) {
    const int T = (int)std::min<int64_t>(n_threads(), std::max<int64_t>(n, 1));
    std::atomic<int64_t> next{0};
    auto work = [&]() {
        for (int64_t i; (i = next.fetch_add(1)) < n;) fn(i);
    };
    std::vector<std::thread> th;
    for (int k = 1; k < T; ++k) th.emplace_back(work);
    work();
    for (auto &w : th) w.join();
}

constexpr int64_t kNoiseChunk = 1 << 20;

// The stream's plan (pass 1): bars, simulated step count, and the number of
// events per microsecond of stamp offset and per column (before the tail cut).
struct Stream {
    farms_synth_params p{};
    std::vector<Bar> bars;
    int64_t n_noise = 0, n_signal = 0;
    uint32_t steps = 0;        // signal time steps simulated
    uint64_t span_us = 1;      // noise stamps are uniform in [0, span)
    std::vector<uint32_t> ht;  // events per us offset (length: horizon)
    std::vector<int64_t> hx;   // events per column
    std::vector<int64_t> cum;  // cum[b] = events with t_off < b (length ht.size() + 1)
    uint64_t noise_seed = 0;
};

inline void noise_event(const Stream &S, int64_t k, uint32_t &t_off, int &x, int &y, int &p) {
    const uint64_t z = mix64(S.noise_seed + (uint64_t)k * 0xD1B54A32D192ED03ull);
    t_off = (uint32_t)(z % S.span_us);
    x = (int)(mix64(z ^ 1) % (uint64_t)S.p.width);
    y = (int)(mix64(z ^ 2) % (uint64_t)S.p.height);
    p = (mix64(z ^ 3) & 1) ? +1 : -1;
}

int plan_stream(const farms_synth_params *p, Stream &S) {
    if (!p || p->width <= 0 || p->height <= 0 || p->width > 65535 || p->height > 32767 ||
        p->n_events < 0 || p->n_bars < 0 || p->noise_frac < 0 || p->noise_frac >= 1 || p->jitter_us < 0)
        return -1;
    if (p->n_events > 0 && p->n_bars == 0 && p->noise_frac <= 0) return -1;
    S.p = *p;
    const int W = p->width, H = p->height, J = p->jitter_us;
    SplitMix64 rng(p->seed);
    S.bars.resize((size_t)p->n_bars);
    for (Bar &b : S.bars) {
        b.cx = rng.uniform(0, W - 1);
        b.cy = rng.uniform(0, H - 1);
        double dir;
        if (p->fixed_dir_deg >= 0) {
            dir = p->fixed_dir_deg * kPi / 180.0;
        } else {  // reject directions within 10 degrees of an axis
            do { dir = rng.uniform(0, 2 * kPi); } while (std::fmod(dir, kPi / 2) < 10 * kPi / 180 ||
                                                         std::fmod(dir, kPi / 2) > 80 * kPi / 180);
        }
        double speed = rng.uniform(p->speed_min, p->speed_max);
        b.vx = speed * std::cos(dir);
        b.vy = speed * std::sin(dir);
        double axis = dir + kPi / 2 + (p->fixed_dir_deg >= 0 ? 0.0 : rng.uniform(-20, 20) * kPi / 180);
        b.ux = std::cos(axis); b.uy = std::sin(axis);
        b.mx = -b.uy; b.my = b.ux;
        b.half_len = 0.5 * rng.uniform(p->len_min, p->len_max);
        b.half_thick = 0.5 * rng.uniform(p->thick_min, p->thick_max);
    }
    S.noise_seed = rng.next();
    S.n_noise = (int64_t)std::llround((double)p->n_events * p->noise_frac);
    S.n_signal = p->n_events - S.n_noise;
    S.hx.assign((size_t)W, 0);
    S.ht.clear();
    const int64_t target = S.n_signal > 0 && !S.bars.empty() ? S.n_signal + S.n_signal / 64 + 1024 : 0;
    // signal: rounds of blocks of kBlockSteps steps on parallel threads, each
    // with local per-step / per-us / per-column counts, merged in block order
    // until the step where the simulated signal reaches the target
    const int nb = 4 * n_threads();
    const uint32_t blk_us = kBlockSteps * kStepUs + (uint32_t)J + 1;  // stamp offsets of one block
    struct Blk {
        uint32_t s0;
        std::vector<Bar> st;
        std::vector<int64_t> per_step, hx;
        std::vector<uint32_t> ht;
    };
    std::vector<Blk> blk((size_t)nb);
    auto count_block = [&](Blk &B, uint32_t s_end) {
        B.per_step.assign(kBlockSteps, 0);
        B.ht.assign(blk_us, 0);
        B.hx.assign((size_t)W, 0);
        std::vector<Bar> bars = B.st;
        for (uint32_t s = B.s0; s < s_end; ++s) {
            int64_t cnt = 0;
            for (size_t bi = 0; bi < bars.size(); ++bi)
                emit_bar_step(bars[bi], (int)bi, s, W, H, J, p->seed, [&](uint32_t tt, int px, int, int) {
                    ++cnt;
                    B.ht[tt - B.s0 * kStepUs]++;
                    B.hx[(size_t)px]++;
                });
            B.per_step[s - B.s0] = cnt;
            advance(bars, W, H);
        }
    };
    std::vector<Bar> cur = S.bars;
    int64_t have = 0;
    uint32_t s_base = 0;
    bool done = target == 0;
    while (!done) {
        if ((uint64_t)s_base + (uint64_t)nb * kBlockSteps > 4000000000ull / kStepUs) return -2;  // uint32 time
        for (int i = 0; i < nb; ++i) {
            blk[(size_t)i].s0 = s_base + (uint32_t)i * kBlockSteps;
            blk[(size_t)i].st = cur;
            for (int s = 0; s < kBlockSteps; ++s) advance(cur, W, H);
        }
        parallel_for(nb, [&](int64_t i) { count_block(blk[(size_t)i], blk[(size_t)i].s0 + kBlockSteps); });
        for (int i = 0; i < nb && !done; ++i) {
            Blk &B = blk[(size_t)i];
            int s_stop = kBlockSteps;
            for (int s = 0; s < kBlockSteps; ++s) {
                have += B.per_step[(size_t)s];
                if (have >= target) { s_stop = s + 1; done = true; break; }
            }
            if (s_stop < kBlockSteps) count_block(B, B.s0 + (uint32_t)s_stop);  // the last steps only
            const size_t need = (size_t)B.s0 * kStepUs + blk_us;
            if (S.ht.size() < need) S.ht.resize(need, 0);
            for (uint32_t u = 0; u < blk_us; ++u) S.ht[(size_t)B.s0 * kStepUs + u] += B.ht[u];
            for (int x = 0; x < W; ++x) S.hx[(size_t)x] += B.hx[(size_t)x];
            S.steps = B.s0 + (uint32_t)s_stop;
        }
        s_base += (uint32_t)nb * kBlockSteps;
    }
    S.span_us = std::max<uint64_t>(1, (uint64_t)S.steps * kStepUs);
    if (S.ht.size() < S.span_us) S.ht.resize(S.span_us, 0);
    // noise: counter-based draws, counted with atomic adds
    {
        std::vector<std::atomic<int64_t>> hx(W);
        for (auto &v : hx) v.store(0);
        uint32_t *ht = S.ht.data();
        const int64_t nchunks = (S.n_noise + kNoiseChunk - 1) / kNoiseChunk;
        parallel_for(nchunks, [&](int64_t c) {
            std::vector<int64_t> lx((size_t)W, 0);
            const int64_t k1 = std::min(S.n_noise, (c + 1) * kNoiseChunk);
            for (int64_t k = c * kNoiseChunk; k < k1; ++k) {
                uint32_t t; int x, y, pp;
                noise_event(S, k, t, x, y, pp);
                __atomic_fetch_add(&ht[t], 1u, __ATOMIC_RELAXED);
                lx[(size_t)x]++;
            }
            for (int x = 0; x < W; ++x) hx[(size_t)x].fetch_add(lx[(size_t)x]);
        });
        for (int x = 0; x < W; ++x) S.hx[(size_t)x] += hx[(size_t)x].load();
    }
    S.cum.assign(S.ht.size() + 1, 0);
    for (size_t b = 0; b < S.ht.size(); ++b) S.cum[b + 1] = S.cum[b] + S.ht[b];
    if (S.cum.back() < p->n_events) return -3;
    return 0;
}

// Pass 2: the keys with stamp offset in [ta, tb] and column in [x_lo, x_hi),
// sorted; below[t - ta] (if given) counts the events of that microsecond in
// columns < x_lo.
void collect(const Stream &S, uint32_t ta, uint32_t tb, int x_lo, int x_hi, std::vector<uint64_t> &keys,
             std::vector<uint32_t> *below) {
    const int W = S.p.width, H = S.p.height, J = S.p.jitter_us;
    const uint32_t t0 = S.p.t0;
    if (below) below->assign((size_t)(tb - ta) + 1, 0);
    uint32_t *bl = below ? below->data() : nullptr;
    auto keep = [&](std::vector<uint64_t> &out, uint32_t tt, int px, int py, int pol) {
        if (tt < ta || tt > tb) return;
        if (px < x_lo) {
            if (bl) __atomic_fetch_add(&bl[tt - ta], 1u, __ATOMIC_RELAXED);
            return;
        }
        if (px >= x_hi) return;
        out.push_back(make_key(t0 + tt, px, py, pol));
    };
    const int64_t nblk = ((int64_t)S.steps + kBlockSteps - 1) / kBlockSteps;
    const int64_t nchunks = (S.n_noise + kNoiseChunk - 1) / kNoiseChunk;
    std::vector<std::vector<uint64_t>> part((size_t)(nblk + nchunks));
    // bar states at each block start (sequential, cheap)
    std::vector<std::vector<Bar>> st((size_t)nblk);
    {
        std::vector<Bar> cur = S.bars;
        for (int64_t i = 0; i < nblk; ++i) {
            st[(size_t)i] = cur;
            for (int s = 0; s < kBlockSteps; ++s) advance(cur, W, H);
        }
    }
    parallel_for(nblk + nchunks, [&](int64_t i) {
        std::vector<uint64_t> &out = part[(size_t)i];
        if (i < nblk) {
            const uint32_t s0 = (uint32_t)i * kBlockSteps;
            const uint32_t s1 = std::min<uint32_t>(S.steps, s0 + kBlockSteps);
            if ((uint64_t)s0 * kStepUs > tb || (uint64_t)s1 * kStepUs + (uint64_t)J < ta) return;  // outside the window
            std::vector<Bar> bars = st[(size_t)i];
            for (uint32_t s = s0; s < s1; ++s) {
                for (size_t bi = 0; bi < bars.size(); ++bi)
                    emit_bar_step(bars[bi], (int)bi, s, W, H, J, S.p.seed,
                                  [&](uint32_t tt, int px, int py, int pol) { keep(out, tt, px, py, pol); });
                advance(bars, W, H);
            }
        } else {
            const int64_t c = i - nblk;
            const int64_t k1 = std::min(S.n_noise, (c + 1) * kNoiseChunk);
            for (int64_t k = c * kNoiseChunk; k < k1; ++k) {
                uint32_t t; int x, y, pp;
                noise_event(S, k, t, x, y, pp);
                keep(out, t, x, y, pp);
            }
        }
    });
    size_t total = 0;
    for (auto &v : part) total += v.size();
    keys.clear();
    keys.reserve(total);
    for (auto &v : part) {
        keys.insert(keys.end(), v.begin(), v.end());
        std::vector<uint64_t>().swap(v);
    }
    radix_sort_u64(keys);
}

inline void unpack(uint64_t k, int32_t &x, int32_t &y, uint32_t &t, int32_t &pol) {
    t = (uint32_t)(k >> 32);
    x = (int32_t)((k >> 16) & 0xFFFF);
    y = (int32_t)((k >> 1) & 0x7FFF);
    pol = (k & 1) ? 1 : -1;
}

// The microsecond bucket holding stream index e (0 <= e < cum.back()).
uint32_t bucket_of(const Stream &S, int64_t e) {
    return (uint32_t)(std::upper_bound(S.cum.begin(), S.cum.end(), e) - S.cum.begin() - 1);
}

}  // namespace

extern "C" int farms_synth_preset(int config, farms_synth_params *o) {
    if (!o) return -1;
    std::memset(o, 0, sizeof(*o));
    o->t0 = 1000000u;
    o->fixed_dir_deg = -1.0;
    o->jitter_us = 20;
    o->noise_frac = 0.05;
    switch (config) {
    case 1:  // 128x128, 100k events, 1 bar L=60 w=5 dir 30 deg |v|=500
        o->width = 128; o->height = 128; o->n_events = 100000; o->n_bars = 1;
        o->len_min = o->len_max = 60; o->thick_min = o->thick_max = 5;
        o->speed_min = o->speed_max = 500; o->jitter_us = 15; o->noise_frac = 0.02;
        o->fixed_dir_deg = 30.0; o->seed = 0x5EED0001ull;
        return 0;
    case 2:  // 320x320 ATIS-shape, 2M events, 8 bars
        o->width = 320; o->height = 320; o->n_events = 2000000; o->n_bars = 8;
        o->len_min = 40; o->len_max = 120; o->thick_min = 3; o->thick_max = 8;
        o->speed_min = 200; o->speed_max = 1500; o->seed = 0x5EED0002ull;
        return 0;
    case 3: case 4: case 5:  // 1280x720 DVS-shape, 64 bars
        o->width = 1280; o->height = 720; o->n_bars = 64;
        o->len_min = 60; o->len_max = 300; o->thick_min = 3; o->thick_max = 10;
        o->speed_min = 300; o->speed_max = 3000;
        o->n_events = config == 3 ? 50000000ll : config == 4 ? 200000000ll : 1000000000ll;
        o->seed = config == 3 ? 0x5EED0003ull : config == 4 ? 0x5EED0004ull : 0x5EED0005ull;
        return 0;
    default:
        return -1;
    }
}

extern "C" int64_t farms_synth_generate(const farms_synth_params *p, int32_t *x, int32_t *y,
                                        uint32_t *t, int32_t *pol) {
    return farms_synth_generate_select(p, 0, p ? p->n_events : 0, 0, p ? p->width : 0, p ? p->n_events : 0, x, y, t,
                                       pol, nullptr, nullptr);
}

extern "C" int64_t farms_synth_generate_select(const farms_synth_params *p, int64_t e0, int64_t e1,
                                               int32_t x_lo, int32_t x_hi, int64_t cap, int32_t *x,
                                               int32_t *y, uint32_t *t, int32_t *pol, int64_t *idx,
                                               uint32_t *t_first) {
    if (!p || e0 < 0 || e1 < e0 || cap < 0 || (cap > 0 && (!x || !y || !t || !pol))) return -1;
    Stream S;
    int rc = plan_stream(p, S);
    if (rc) return rc;
    const int64_t n = p->n_events;
    if (t_first) *t_first = n > 0 ? p->t0 + bucket_of(S, 0) : 0u;
    if (e1 > n) e1 = n;
    x_lo = std::max(x_lo, 0);
    x_hi = std::min(x_hi, p->width);
    if (e0 >= e1 || x_lo >= x_hi) return 0;
    const uint32_t ta = bucket_of(S, e0), tb = bucket_of(S, e1 - 1);
    const bool all_cols = x_lo == 0 && x_hi == p->width;
    std::vector<uint64_t> keys;
    std::vector<uint32_t> below;
    collect(S, ta, tb, x_lo, x_hi, keys, all_cols ? nullptr : &below);
    // stream index of each kept key: the events of earlier microseconds, the
    // earlier columns of its own microsecond, its rank among the kept ones
    int64_t m = 0;
    size_t k = 0;
    while (k < keys.size()) {
        const uint32_t b = (uint32_t)(keys[k] >> 32) - p->t0;
        const int64_t base = S.cum[b] + (all_cols ? 0 : (int64_t)below[b - ta]);
        size_t j = k;
        for (; j < keys.size() && (uint32_t)(keys[j] >> 32) - p->t0 == b; ++j) {
            const int64_t e = base + (int64_t)(j - k);
            if (e < e0 || e >= e1) continue;
            if (m < cap) {
                unpack(keys[j], x[m], y[m], t[m], pol[m]);
                if (idx) idx[m] = e;
            }
            ++m;
        }
        k = j;
    }
    return m;
}

extern "C" int farms_synth_write_text(const char *path, const int32_t *x, const int32_t *y,
                                      const uint32_t *t, const int32_t *pol, int64_t n) {
    FILE *f = std::fopen(path, "wb");
    if (!f) return -1;
    std::vector<char> buf(1 << 20);
    size_t used = 0;
    for (int64_t e = 0; e < n; ++e) {
        if (buf.size() - used < 64) { std::fwrite(buf.data(), 1, used, f); used = 0; }
        used += (size_t)std::snprintf(buf.data() + used, 64, "%d %d %u %d\n", x[e], y[e], t[e], pol[e]);
    }
    std::fwrite(buf.data(), 1, used, f);
    return std::fclose(f) == 0 ? 0 : -1;
}

extern "C" int farms_synth_column_hist(const farms_synth_params *p, int64_t *hist) {
    if (!p || !hist) return -1;
    Stream S;
    int rc = plan_stream(p, S);
    if (rc) return rc;
    for (int x = 0; x < p->width; ++x) hist[x] = S.hx[(size_t)x];
    // minus the tail cut: events with stream index >= n_events
    const int64_t n = p->n_events, total = S.cum.back();
    if (total > n) {
        const uint32_t ta = bucket_of(S, n), tb = (uint32_t)S.ht.size() - 1;
        std::vector<uint64_t> keys;
        collect(S, ta, tb, 0, p->width, keys, nullptr);
        for (size_t j = 0; j < keys.size(); ++j)
            if (S.cum[ta] + (int64_t)j >= n) hist[key_x(keys[j])]--;
    }
    return 0;
}
