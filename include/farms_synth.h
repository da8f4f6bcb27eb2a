/*
 * farms_synth.h — seeded synthetic DVS/ATIS event streams ("moving bars").
 *
 * Workload generator for the parity tests and bench.py.  The
 * reference ships no sample data, so every stream used here is
 * produced by this generator from a documented seed.  Host-only C ABI.
 *
 * Model: each bar is a bright rectangle (long side L, thickness w) moving at a
 * constant velocity and reflecting at the sensor border.  A pixel centre that
 * enters the rectangle fires p=+1, one that leaves it fires p=-1, at the exact
 * crossing instant (piecewise-linear motion in 100 us steps), plus U{0..J} us of
 * jitter.  A fraction of uniform background-noise events is mixed in.  Events
 * are sorted by (t, x, y, p); t is absolute microseconds starting at t0.
 * PRNG: SplitMix64 (documented in farms_synth.cpp).
 */
#ifndef FARMS_SYNTH_H
#define FARMS_SYNTH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int32_t width, height;
    int64_t n_events;      /* exact number of events to emit */
    int32_t n_bars;
    double len_min, len_max;     /* bar length L, px */
    double thick_min, thick_max; /* bar thickness w, px */
    double speed_min, speed_max; /* |v|, px/s */
    int32_t jitter_us;           /* timing jitter U{0..J} */
    double noise_frac;           /* fraction of all events that are uniform noise */
    uint64_t seed;
    uint32_t t0;                 /* first possible timestamp, us */
    double fixed_dir_deg;        /* >= 0: every bar moves in this direction (config 1) */
} farms_synth_params;

/* Fill `out` with BASELINE.json configuration `config` (1..5).
 * Returns 0, or -1 for an unknown config. */
int farms_synth_preset(int config, farms_synth_params *out);

/* Generate exactly p->n_events events into caller-owned arrays of that length.
 * Returns the number of events written (== n_events), or a negative code. */
int64_t farms_synth_generate(const farms_synth_params *p, int32_t *x, int32_t *y,
                             uint32_t *t, int32_t *pol);

/* The events with index in [e0, e1) and column in [x_lo, x_hi) of the stream
 * farms_synth_generate would produce, in stream order, with their stream
 * indices in idx (may be NULL), and the stream's first stamp in *t_first (may
 * be NULL; the t0 of vFlow.cpp:194): one rank's share of a multi-GPU run
 * without holding the whole stream.  At most cap events are written; returns
 * how many events match (possibly > cap), or a negative code. */
int64_t farms_synth_generate_select(const farms_synth_params *p, int64_t e0, int64_t e1,
                                    int32_t x_lo, int32_t x_hi, int64_t cap, int32_t *x,
                                    int32_t *y, uint32_t *t, int32_t *pol, int64_t *idx,
                                    uint32_t *t_first);

/* Events per column (p->width counts) of the whole stream: the balance of a
 * multi-GPU x-strip plan.  Returns 0 or a negative code. */
int farms_synth_column_hist(const farms_synth_params *p, int64_t *hist);

/* Write events as the reference's input text format, one "x y t p" line per
 * event (README.md "Input event files").  Returns 0 or -1 on I/O error. */
int farms_synth_write_text(const char *path, const int32_t *x, const int32_t *y,
                           const uint32_t *t, const int32_t *pol, int64_t n);

#ifdef __cplusplus
}
#endif
#endif
