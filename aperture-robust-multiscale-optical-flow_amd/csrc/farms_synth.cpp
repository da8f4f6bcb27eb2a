// farms_synth.cpp — seeded "moving bars" event-stream generator.
//
// Workload tool for tests and bench.py; not part of the accelerated path.  The
// reference ships no data, so the configurations of BASELINE.json
// are synthesised here from documented seeds.
//
// PRNG: SplitMix64 (Steele, Lea, Flood 2014):
//   s += 0x9E3779B97F4A7C15; z = s; z = (z ^ z>>30) * 0xBF58476D1CE4E5B9;
//   z = (z ^ z>>27) * 0x94D049BB133111EB; return z ^ z>>31;
// uniform double = (z >> 11) * 2^-53.
//
// Geometry: pixel (px, py) has its centre at (px, py).  A bar is the rectangle
// |(q-c).u| <= L/2, |(q-c).m| <= w/2 with u the long axis and m its normal.  The
// centre moves with constant velocity inside each 100 us step and reflects off
// the sensor border between steps.  For every edge of the rectangle the pixels
// of its swept parallelogram are visited by scanline and the exact entry (ON,
// p=+1) / exit (OFF, p=-1) instant of each pixel centre is solved from the two
// slab intervals; an event is emitted by the edge that binds it, so corners are
// not duplicated.
#include "../../include/farms_synth.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
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
    uint64_t below(uint64_t n) { return n ? next() % n : 0; }
};

constexpr double kPi = 3.14159265358979323846;
constexpr double kStepUs = 100.0;  // motion is linear within a step
constexpr double kStepS = kStepUs * 1e-6;

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

void emit_bar_step(const Bar &b, uint32_t step_t0_us, int W, int H, int jitter, SplitMix64 &rng,
                   std::vector<uint64_t> &keys, uint32_t t0) {
    const double vu = b.vx * b.ux + b.vy * b.uy;
    const double vm = b.vx * b.mx + b.vy * b.my;
    const V2 dv{b.vx * kStepS, b.vy * kStepS};
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
                        uint32_t tt = t0 + step_t0_us + (uint32_t)std::floor(tau * 1e6) +
                                      (uint32_t)rng.below((uint64_t)jitter + 1);
                        keys.push_back(make_key(tt, px, py, which == 0 ? +1 : -1));
                    }
                }
            }
        }
    }
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

namespace {

// The whole stream as sorted keys (at least n_events of them), or a negative code.
int64_t generate_keys(const farms_synth_params *p, std::vector<uint64_t> &keys) {
    if (!p || p->width <= 0 || p->height <= 0 || p->width > 65535 || p->height > 32767 ||
        p->n_events < 0 || p->n_bars < 0 || p->noise_frac < 0 || p->noise_frac >= 1)
        return -1;
    if (p->n_events == 0) return 0;
    if (p->n_bars == 0 && p->noise_frac <= 0) return -1;
    const int W = p->width, H = p->height;
    SplitMix64 rng(p->seed);
    std::vector<Bar> bars((size_t)p->n_bars);
    for (Bar &b : bars) {
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
    const int64_t n_noise = (int64_t)std::llround((double)p->n_events * p->noise_frac);
    const int64_t n_signal = p->n_events - n_noise;
    keys.clear();
    keys.reserve((size_t)(p->n_events + p->n_events / 16 + 4096));
    // simulate until the signal budget (plus a margin for the tail cut) is reached
    const int64_t margin = n_signal / 64 + 1024;
    uint32_t step = 0;
    if (n_signal > 0 && !bars.empty()) {
        while ((int64_t)keys.size() < n_signal + margin) {
            for (Bar &b : bars) {
                emit_bar_step(b, step * (uint32_t)kStepUs, W, H, p->jitter_us, rng, keys, p->t0);
                b.cx += b.vx * kStepS;
                b.cy += b.vy * kStepS;
                if (b.cx < 0) { b.cx = -b.cx; b.vx = -b.vx; }
                if (b.cx > W - 1) { b.cx = 2.0 * (W - 1) - b.cx; b.vx = -b.vx; }
                if (b.cy < 0) { b.cy = -b.cy; b.vy = -b.vy; }
                if (b.cy > H - 1) { b.cy = 2.0 * (H - 1) - b.cy; b.vy = -b.vy; }
            }
            ++step;
            if (step > 4000000000u / (uint32_t)kStepUs) return -2;  // would overflow uint32 time
        }
    }
    const uint64_t span_us = std::max<uint64_t>(1, (uint64_t)step * (uint64_t)kStepUs);
    for (int64_t k = 0; k < n_noise; ++k) {
        uint32_t tt = p->t0 + (uint32_t)rng.below(span_us);
        int nx = (int)rng.below((uint64_t)W), ny = (int)rng.below((uint64_t)H);
        keys.push_back(make_key(tt, nx, ny, (rng.next() & 1) ? +1 : -1));
    }
    radix_sort_u64(keys);
    if ((int64_t)keys.size() < p->n_events) return -3;
    return p->n_events;
}

inline void unpack(uint64_t k, int32_t &x, int32_t &y, uint32_t &t, int32_t &pol) {
    t = (uint32_t)(k >> 32);
    x = (int32_t)((k >> 16) & 0xFFFF);
    y = (int32_t)((k >> 1) & 0x7FFF);
    pol = (k & 1) ? 1 : -1;
}

}  // namespace

extern "C" int64_t farms_synth_generate(const farms_synth_params *p, int32_t *x, int32_t *y,
                                        uint32_t *t, int32_t *pol) {
    std::vector<uint64_t> keys;
    const int64_t n = generate_keys(p, keys);
    if (n <= 0) return n;
    for (int64_t e = 0; e < n; ++e) unpack(keys[(size_t)e], x[e], y[e], t[e], pol[e]);
    return n;
}

extern "C" int64_t farms_synth_generate_select(const farms_synth_params *p, int64_t e0, int64_t e1,
                                               int32_t x_lo, int32_t x_hi, int64_t cap, int32_t *x,
                                               int32_t *y, uint32_t *t, int32_t *pol, int64_t *idx,
                                               uint32_t *t_first) {
    if (!p || e0 < 0 || e1 < e0 || cap < 0 || (cap > 0 && (!x || !y || !t || !pol))) return -1;
    std::vector<uint64_t> keys;
    const int64_t n = generate_keys(p, keys);
    if (n < 0) return n;
    if (t_first) *t_first = n > 0 ? (uint32_t)(keys[0] >> 32) : 0u;
    if (e1 > n) e1 = n;
    int64_t m = 0;
    for (int64_t e = e0; e < e1; ++e) {
        const uint64_t k = keys[(size_t)e];
        const int32_t kx = (int32_t)((k >> 16) & 0xFFFF);
        if (kx < x_lo || kx >= x_hi) continue;
        if (m < cap) {
            unpack(k, x[m], y[m], t[m], pol[m]);
            if (idx) idx[m] = e;
        }
        ++m;
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
    std::vector<uint64_t> keys;
    const int64_t n = generate_keys(p, keys);
    if (n < 0) return (int)n;
    std::memset(hist, 0, sizeof(int64_t) * (size_t)p->width);
    for (int64_t e = 0; e < n; ++e) hist[(keys[(size_t)e] >> 16) & 0xFFFF]++;
    return 0;
}
