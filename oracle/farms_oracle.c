/*
 * farms_oracle.c — CPU restatement of the FARMS_Flow batch hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see farms_oracle.h).  Status: "parity unpinned" —
 * no reference fixtures exist and the reference is unbuildable here.
 *
 * Deliberately "reference-shaped": dense nested loops over the same surfaces in
 * the same order as /root/reference/src/vFlow.cpp, single thread, fp64, no FMA
 * (build with -ffp-contract=off), so it doubles as the timed CPU baseline.
 * Eigen calls are restated from Eigen 3.4 semantics (the libeigen3-dev the
 * reference README asks for on this image's Ubuntu 22.04), see DESIGN.md §3.
 *
 * Deviations from the reference, all documented in DESIGN.md:
 *   - pooling cells whose x-major linear index is >= W*H (reference: read past
 *     the end of the vector, undefined behaviour, vFlow.cpp:1000/1113 with the
 *     last column) are treated as non-contributing;
 *   - pow(v, 2.0) (vFlow.cpp:1349) is evaluated as v*v, what g++ -O2 emits;
 *   - events outside the sensor are rejected instead of corrupting the heap.
 */
#include "farms_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define MAXSTAMP 4294967296.0 /* vFlow.h:27  pow(2, 32) */
#define TSTOSEC 1e-6          /* vFlow.h:28 */
#define KILL_OLD_FLOW_TIME 500.0 /* vFlow.cpp:961 */

struct farms_oracle {
    int W, H;
    int serial; /* vFlowManager::run semantics (farms_oracle.h) */
    int eigen;  /* 34 (default) or 33: the Eigen version whose GEMV order (A2*At)*Y follows (farms_oracle_set_eigen) */
    /* libm of the path: glibc's atan2 / sin / cos (the reference's) unless a
     * test swaps in another implementation (farms_oracle_set_libm) */
    double (*f_atan2)(double, double);
    double (*f_sin)(double);
    double (*f_cos)(double);
    int frad, plane_size, min_inliers;
    int window_jump, max_window, nscales;
    /* cSurf (vFlow.h:51): stored Event x, y, stamp per cell, x-major (EventMatrix.h:32-33) */
    int *cs_x, *cs_y;
    double *cs_t;
    double *last_time;  /* lastEventTime (vFlow.h:73) */
    double *flow_len;   /* flowSurfaceLengthOn/Of (identical, vFlow.cpp:349-353) */
    double *flow_theta; /* flowSurfaceThetaOn/Of */
    /* computeTrueFlow scratch (vFlow.cpp:966-977) */
    double *pool, *pool_x, *pool_y;
    double *scratch; /* computeGrads A/Y rows and one row's products: 5 * planeSize doubles */
};

int farms_oracle_create(int width, int height, int filter_size, int min_inliers,
                        int window_jump, int max_window, farms_oracle **out)
{
    if (!out || width <= 0 || height <= 0 || window_jump <= 0 || max_window < 0) return -1;
    /* vFlow.cpp:32-36: fs < 5 -> 3; even -> fs-1; fRad = fs/2; planeSize = fs^2 */
    if (filter_size < 5) filter_size = 3;
    if (!(filter_size % 2)) filter_size--;
    int nscales = max_window / window_jump + 1;
    /* spatialPool is vector<double>(maxWindow) indexed with .at(numWindows)
     * (vFlow.cpp:966,1025): more scales than maxWindow throws in the reference. */
    if (nscales > max_window) return -1;
    farms_oracle *o = (farms_oracle *)calloc(1, sizeof(*o));
    if (!o) return -3;
    o->W = width;
    o->H = height;
    o->frad = filter_size / 2;
    o->plane_size = filter_size * filter_size;
    o->min_inliers = min_inliers;
    o->window_jump = window_jump;
    o->max_window = max_window;
    o->nscales = nscales;
    o->eigen = 34;
    o->f_atan2 = atan2;
    o->f_sin = sin;
    o->f_cos = cos;
    size_t cells = (size_t)width * (size_t)height;
    o->cs_x = (int *)calloc(cells, sizeof(int));
    o->cs_y = (int *)calloc(cells, sizeof(int));
    o->cs_t = (double *)calloc(cells, sizeof(double));
    o->last_time = (double *)calloc(cells, sizeof(double));
    o->flow_len = (double *)calloc(cells, sizeof(double));
    o->flow_theta = (double *)calloc(cells, sizeof(double));
    o->pool = (double *)calloc((size_t)nscales, sizeof(double));
    o->pool_x = (double *)calloc((size_t)nscales, sizeof(double));
    o->pool_y = (double *)calloc((size_t)nscales, sizeof(double));
    o->scratch = (double *)calloc(5 * (size_t)o->plane_size, sizeof(double));
    if (!o->scratch || !o->cs_x || !o->cs_y || !o->cs_t || !o->last_time || !o->flow_len || !o->flow_theta ||
        !o->pool || !o->pool_x || !o->pool_y) {
        farms_oracle_destroy(o);
        return -3;
    }
    *out = o;
    return 0;
}

void farms_oracle_destroy(farms_oracle *o)
{
    if (!o) return;
    free(o->cs_x); free(o->cs_y); free(o->cs_t); free(o->last_time);
    free(o->flow_len); free(o->flow_theta);
    free(o->pool); free(o->pool_x); free(o->pool_y); free(o->scratch);
    free(o);
}

int farms_oracle_num_scales(const farms_oracle *o) { return o ? o->nscales : 0; }

/* SAE seed for temporal-segment tests: a visited cell holds Event(x, y, p, t)
 * and lastEventTime t (vFlow.cpp:264,267), an unvisited one Event(0,0,0,0). */
void farms_oracle_seed_sae(farms_oracle *o, const int64_t *stamp)
{
    const int W = o->W, H = o->H;
    for (int x = 0; x < W; ++x)
        for (int y = 0; y < H; ++y) {
            const size_t c = (size_t)x * H + y;
            const int vis = stamp[c] >= 0;
            o->cs_x[c] = vis ? x : 0;
            o->cs_y[c] = vis ? y : 0;
            o->cs_t[c] = vis ? (double)stamp[c] : 0.0;
            o->last_time[c] = vis ? (double)stamp[c] : 0.0;
        }
}

/* ---- Eigen 3.4 restatements ------------------------------------------------ */

/* AtA.determinant() on a MatrixXd (vFlow.cpp:1316).  A dynamic-size matrix goes
 * through PartialPivLU: unblocked LU (size <= 16), pivot = FIRST row holding the
 * largest |a_ik| (strict >), row swap counted, column tail divided by the pivot,
 * trailing update a_ij -= l_i * u_j; det = (+-1) * ((u00*u11)*u22).
 * `ata` is column-major as AtA.data() (vFlow.cpp:1315). */
static double eigen_det3_partialpivlu(const double ata[9])
{
    double m[3][3];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) m[r][c] = ata[c * 3 + r];
    int transpositions = 0;
    for (int k = 0; k < 3; ++k) {
        int piv = k;
        double big = fabs(m[k][k]);
        for (int i = k + 1; i < 3; ++i) {
            double s = fabs(m[i][k]);
            if (s > big) { big = s; piv = i; }
        }
        if (big != 0.0) {
            if (piv != k) {
                for (int c = 0; c < 3; ++c) { double tmp = m[k][c]; m[k][c] = m[piv][c]; m[piv][c] = tmp; }
                ++transpositions;
            }
            for (int i = k + 1; i < 3; ++i) m[i][k] = m[i][k] / m[k][k];
        }
        for (int i = k + 1; i < 3; ++i)
            for (int j = k + 1; j < 3; ++j) m[i][j] = m[i][j] - m[i][k] * m[k][j];
    }
    double prod = (m[0][0] * m[1][1]) * m[2][2];
    return (transpositions & 1) ? -prod : prod;
}

/* Eigen 3.3's column-major GEMV (GeneralMatrixVector.h, as published in the
 * 3.3 series; the 3.4 rewrite accumulates every row sequentially from zero) for
 * temp = (A2*At) * Y, the 3 x n temporary times the n x 1 runtime vector Y
 * (vFlow.cpp:1338), with SSE2 packets of 2 doubles, for one of the two packet
 * rows (rows 0 and 1: a and b; row 2, the intercept c, is a scalar remainder
 * row and is never used by the reference).  The destination starts at zero
 * (dst.setZero()) and is 16-B aligned, so rows 0-1 form the one aligned packet;
 * the temporary's column stride is 3 (odd), so alignmentStep = 1 and the
 * kernel's offset1 / offset3 swap (its `FirstAligned && alignmentStep==1` test
 * reads the enum constant): each block of 4 columns i..i+3 takes lhs0..lhs3 =
 * columns i, i+3, i+2, i+1 and _EIGEN_ACCUMULATE_PACKETS adds
 *     res = res + ((p[i] + p[i+3]) + (p[i+2] + p[i+1]));
 * the n % 4 remaining columns follow one at a time (res = res + p[k]).  p[k] is
 * (A2*At)(r, k) * Y(k) (alpha = 1: exact).  Only the order of the additions
 * differs from 3.4; whether it changes a record is measured, not assumed
 * (tools/eigen_sensitivity.py). */
static double eigen33_gemv_packet_row(const double *p, int n)
{
    double res = 0.0;
    const int bound = n / 4 * 4;
    for (int i = 0; i < bound; i += 4) res = res + ((p[i] + p[i + 3]) + (p[i + 2] + p[i + 1]));
    for (int k = bound; k < n; ++k) res = res + p[k];
    return res;
}

void farms_oracle_set_eigen(farms_oracle *o, int version)
{
    if (o) o->eigen = version == 33 ? 33 : 34;
}

/* ---- computeGrads (vFlow.cpp:1214-1381) ------------------------------------- */

/* n rows: X[k], Y[k] (stored event coords), T[k] (stored stamp, double).
 * cen = the current event.  Returns the inlier count, writes dtdx/dtdy only when
 * DET >= 1 (vFlow.cpp:1323 returns before touching them otherwise). */
static int compute_grads(const farms_oracle *o, int n, const double *X, const double *Y, const double *T,
                         double cen_x, double cen_y, double cen_t, double *dtdy, double *dtdx,
                         double *Yt /* scratch 2n */)
{
    /* A (n x 3) rows (X, Y, 1); Y = t*1e-6, or (t - 2^32)*1e-6 for stamps in the
     * future of the event (vFlow.cpp:1224-1234). */
    for (int k = 0; k < n; ++k) {
        if (T[k] > cen_t) Yt[k] = (T[k] - MAXSTAMP) * TSTOSEC;
        else Yt[k] = T[k] * TSTOSEC;
    }
    double cx = cen_x, cy = cen_y, cz = cen_t * TSTOSEC; /* vFlow.cpp:1236-1237 */

    /* AtA = At*A (vFlow.cpp:1307-1311): integer-valued, exact in any order. */
    double sxx = 0, sxy = 0, sx = 0, syy = 0, sy = 0, s1 = 0;
    for (int k = 0; k < n; ++k) {
        sxx += X[k] * X[k]; sxy += X[k] * Y[k]; sx += X[k];
        syy += Y[k] * Y[k]; sy += Y[k]; s1 += 1.0;
    }
    const double a[9] = {sxx, sxy, sx, sxy, syy, sy, sx, sy, s1}; /* column-major */
    double DET = eigen_det3_partialpivlu(a);
    if (DET < 1) return 0; /* vFlow.cpp:1323 */

    /* A2 = adjugate / DET with the exact expressions of vFlow.cpp:1327-1336
     * (A2.data() column-major: A2(r,c) = d[c*3+r]). */
    double d[9];
    DET = 1.0 / DET;
    d[0] = DET * (a[8] * a[4] - a[7] * a[5]);
    d[1] = DET * (a[7] * a[2] - a[8] * a[1]);
    d[2] = DET * (a[5] * a[1] - a[4] * a[2]);
    d[3] = DET * (a[6] * a[5] - a[8] * a[3]);
    d[4] = DET * (a[8] * a[0] - a[6] * a[2]);
    d[5] = DET * (a[3] * a[2] - a[5] * a[0]);
    d[6] = DET * (a[7] * a[3] - a[6] * a[4]);
    d[7] = DET * (a[6] * a[1] - a[7] * a[0]);
    d[8] = DET * (a[4] * a[0] - a[3] * a[1]);

    /* temp = A2*At*Y (vFlow.cpp:1338).  Eigen evaluates (A2*At) into a 3 x n
     * temporary, then multiplies by Y.  Both products accumulate in index order:
     *  - A2*At: lazy coefficient product (p0+p1)+p2 when 3+3+n < 20, else GEMM
     *    whose accumulator starts at 0 and is added to a zeroed destination;
     *  - (.)*Y: lazy (first product first) when n+3+1 < 20, else GEMV
     *    (accumulator from 0, then added to a zeroed destination).
     * The two forms differ only in the sign of an all-(-0) sum. */
    const int gemm = (3 + 3 + n) >= 20;
    const int gemv = (n + 3 + 1) >= 20;
    double abc[3];
    for (int r = 0; r < 3; ++r) {
        const double a0 = d[0 * 3 + r], a1 = d[1 * 3 + r], a2 = d[2 * 3 + r];
        double *pr = Yt + n; /* scratch: the n products of row r, (A2*At)(r,k) * Y(k) */
        for (int k = 0; k < n; ++k) {
            double m;
            if (gemm) m = ((((0.0 + a0 * X[k]) + a1 * Y[k]) + a2 * 1.0)) + 0.0;
            else m = (a0 * X[k] + a1 * Y[k]) + a2 * 1.0;
            pr[k] = m * Yt[k];
        }
        if (gemv && o->eigen == 33 && r < 2)
            abc[r] = eigen33_gemv_packet_row(pr, n);
        else {
            double acc = 0.0;
            for (int k = 0; k < n; ++k) {
                if (!gemv && k == 0) acc = pr[k];
                else acc = acc + pr[k];
            }
            abc[r] = gemv ? acc + 0.0 : acc;
        }
    }

    /* vFlow.cpp:1349-1377 */
    double dtdp = sqrt(abc[0] * abc[0] + abc[1] * abc[1]);
    int inliers = 0;
    for (int k = 0; k < n; ++k) {
        double planedt = (abc[0] * (X[k] - cx) + abc[1] * (Y[k] - cy));
        double actualdt = Yt[k] - cz;
        if (fabs(planedt - actualdt) < dtdp / 2 && Yt[k] > 0) inliers++;
    }
    double speed = 1.0 / dtdp;
    double angle = o->f_atan2(abc[0], abc[1]);
    *dtdx = speed * o->f_cos(angle);
    *dtdy = speed * o->f_sin(angle);
    return inliers;
}

/* ---- computeLocalFlow (vFlow.cpp:841-949) ------------------------------------ */

static void compute_local_flow(farms_oracle *o, int ex, int ey, double et, double *vx, double *vy)
{
    const int W = o->W, H = o->H, fr = o->frad, n = o->plane_size;
    double dtdy = 0, dtdx = 0;
    double bestscore = MAXSTAMP + 1;
    int besti = 0, bestj = 0;
    *vx = 0; *vy = 0;
    /* 3 x 3 candidate windows, i outer (vFlow.cpp:870-912) */
    for (int i = ex - fr; i <= ex + fr; i += fr) {
        for (int j = ey - fr; j <= ey + fr; j += fr) {
            int x0 = i - fr < 0 ? 0 : i - fr, x1 = i + fr > W - 1 ? W - 1 : i + fr;
            int y0 = j - fr < 0 ? 0 : j - fr, y1 = j + fr > H - 1 ? H - 1 : j + fr;
            long cnt = (x1 >= x0 && y1 >= y0) ? (long)(x1 - x0 + 1) * (y1 - y0 + 1) : 0;
            if (cnt < n) continue; /* clipped windows are skipped (vFlow.cpp:889) */
            double diff = 0;
            for (int cx = x0; cx <= x1; ++cx)
                for (int cy = y0; cy <= y1; ++cy) {
                    double st = o->cs_t[(size_t)cx * H + cy];
                    diff += et - st;
                    if (st > et) diff += MAXSTAMP;
                }
            diff /= (double)cnt;
            if (diff < bestscore) { bestscore = diff; besti = i; bestj = j; }
        }
    }
    if (bestscore > MAXSTAMP) return; /* vFlow.cpp:915-918 */

    /* gather the winning window cx-major / cy-minor (vFlow.cpp:923-930) */
    double *Xs = o->scratch;
    double *Ys = Xs + n, *Ts = Xs + 2 * n, *Yt = Xs + 3 * n;
    int k = 0;
    for (int cx = (besti - fr < 0 ? 0 : besti - fr); cx <= besti + fr; ++cx)
        for (int cy = (bestj - fr < 0 ? 0 : bestj - fr); cy <= bestj + fr; ++cy) {
            size_t c = (size_t)cx * H + cy;
            Xs[k] = o->cs_x[c];
            Ys[k] = o->cs_y[c];
            Ts[k] = o->cs_t[c];
            ++k;
        }
    int inl = compute_grads(o, k, Xs, Ys, Ts, ex, ey, et, &dtdy, &dtdx, Yt);
    if (inl >= o->min_inliers) { *vx = dtdx; *vy = dtdy; } /* vFlow.cpp:934-942 */
}

/* ---- computeTrueFlow (vFlow.cpp:952-1210; the pol==1 and else branches are
 * the same computation) ------------------------------------------ */

static void compute_true_flow(farms_oracle *o, int x, int y, double te, double *gx, double *gy, int *scale)
{
    const int W = o->W, H = o->H;
    const size_t cells = (size_t)W * H;
    int nw = 0;
    for (int s = 0; s <= o->max_window; s += o->window_jump) {
        double len = 0, sxv = 0, syv = 0, num = 0;
        int i0 = x - s < 0 ? 0 : x - s, i1 = x + s > W - 1 ? W - 1 : x + s;
        int j0 = y - s < 0 ? 0 : y - s, j1 = y + s > W - 1 ? W - 1 : y + s; /* width-1: Q1 */
        for (int i = i0; i <= i1; ++i)
            for (int j = j0; j <= j1; ++j) {
                size_t c = (size_t)i * H + (size_t)j; /* x-major linear index, may alias */
                if (c >= cells) continue;              /* past the end: non-contributing */
                double L = o->flow_len[c];
                if (L > 0 && fabs(te - o->last_time[c]) < KILL_OLD_FLOW_TIME) {
                    len = len + L;
                    sxv = sxv + L * o->f_cos(o->flow_theta[c]);
                    syv = syv + L * o->f_sin(o->flow_theta[c]);
                    num++;
                }
            }
        if (num > 0) { o->pool[nw] = len / num; o->pool_x[nw] = sxv / num; o->pool_y[nw] = syv / num; }
        else { o->pool[nw] = 0; o->pool_x[nw] = 0; o->pool_y[nw] = 0; }
        nw++;
    }
    double maxval = 0;
    int maxi = 0;
    for (int k = 0; k < nw; ++k)
        if (o->pool[k] > maxval) { maxval = o->pool[k]; maxi = k; } /* first strict max */
    if (maxval > 0) {
        *gx = o->pool_x[maxi];
        *gy = o->pool_y[maxi];
        *scale = maxi * o->window_jump;
    } else { /* vFlow.cpp:1085-1094 */
        size_t c = (size_t)x * H + y;
        *gx = o->flow_len[c] * o->f_cos(o->flow_theta[c]);
        *gy = o->flow_len[c] * o->f_sin(o->flow_theta[c]);
        *scale = 0;
    }
}

/* ---- the per-event loop (vFlow.cpp:223-414) ---------------------------------- */

int farms_oracle_process(farms_oracle *o, const int32_t *x, const int32_t *y,
                         const uint32_t *t_rel, const int32_t *p, int64_t n,
                         int32_t *out_x, int32_t *out_y, int32_t *out_t, int32_t *out_p,
                         double *r_true, double *theta_true, double *vx_out, double *vy_out,
                         double *r_local, double *theta_local, int32_t *scale_out)
{
    const int W = o->W, H = o->H;
    for (int64_t e = 0; e < n; ++e)
        if (x[e] < 0 || x[e] >= W || y[e] < 0 || y[e] >= H) return -2;
    for (int64_t e = 0; e < n; ++e) {
        const int ex = x[e], ey = y[e];
        const unsigned int tu = t_rel[e];
        const double et = (double)tu;
        const size_t c = (size_t)ex * H + ey;
        if (!o->serial) o->last_time[c] = et; /* vFlow.cpp:264 (serial: only after pooling, :790) */
        o->cs_x[c] = ex;      /* vFlow.cpp:267 (serial: surfaceOfL, copied to cSurf, :591-610) */
        o->cs_y[c] = ey;
        o->cs_t[c] = et;
        double vx, vy;
        compute_local_flow(o, ex, ey, et, &vx, &vy);
        out_x[e] = ex;
        out_y[e] = ey;
        out_t[e] = (int32_t)tu; /* T_out is vector<int> (vFlow.cpp:136) */
        out_p[e] = p[e];
        vx_out[e] = vx;
        vy_out[e] = vy;
        if (!isnan(fabs(vx)) && !isnan(fabs(vy)) && vx != 0 && vy != 0) { /* vFlow.cpp:315 */
            double length = sqrt(vx * vx + vy * vy);
            double theta = o->f_atan2(vy, vx);
            o->flow_len[c] = length;
            o->flow_theta[c] = theta;
            double gx, gy;
            int sc;
            compute_true_flow(o, ex, ey, et, &gx, &gy, &sc);
            r_true[e] = sqrt(gy * gy + gx * gx);
            theta_true[e] = o->f_atan2(gy, gx);
            r_local[e] = length;
            theta_local[e] = theta;
            scale_out[e] = sc;
        } else {
            r_true[e] = 0; theta_true[e] = 0; r_local[e] = 0; theta_local[e] = 0; scale_out[e] = 0;
            o->flow_len[c] = 0;
            o->flow_theta[c] = 0;
        }
        o->last_time[c] = et; /* vFlow.cpp:407 (serial :790) */
    }
    return 0;
}

void farms_oracle_set_serial(farms_oracle *o, int serial) { o->serial = serial != 0; }

void farms_oracle_set_libm(farms_oracle *o, double (*f_atan2)(double, double), double (*f_sin)(double),
                           double (*f_cos)(double))
{
    o->f_atan2 = f_atan2 ? f_atan2 : atan2;
    o->f_sin = f_sin ? f_sin : sin;
    o->f_cos = f_cos ? f_cos : cos;
}

/* vFlow.cpp:531-556: the first line of the file only stamps lastEventTime, with
 * its absolute time (t0 = time_, the subtraction starts with the next line). */
void farms_oracle_serial_first(farms_oracle *o, int x, int y, uint32_t t_abs)
{
    if (x < 0 || x >= o->W || y < 0 || y >= o->H) return;
    o->last_time[(size_t)x * o->H + y] = (double)t_abs;
}

int farms_oracle_pool_given(farms_oracle *o, const int32_t *x, const int32_t *y, const uint32_t *t_rel,
                            const uint8_t *valid, const double *r_local, const double *theta_local, int64_t n,
                            double *r_true, double *theta_true, int32_t *scale_out)
{
    const int W = o->W, H = o->H;
    for (int64_t e = 0; e < n; ++e)
        if (x[e] < 0 || x[e] >= W || y[e] < 0 || y[e] >= H) return -2;
    for (int64_t e = 0; e < n; ++e) {
        const int ex = x[e], ey = y[e];
        const double et = (double)t_rel[e];
        const size_t c = (size_t)ex * H + ey;
        if (!o->serial) o->last_time[c] = et; /* vFlow.cpp:264 */
        o->cs_x[c] = ex;
        o->cs_y[c] = ey;
        o->cs_t[c] = et;
        if (valid[e]) { /* vFlow.cpp:315-362 with the given (length, theta) */
            o->flow_len[c] = r_local[e];
            o->flow_theta[c] = theta_local[e];
            double gx, gy;
            int sc;
            compute_true_flow(o, ex, ey, et, &gx, &gy, &sc);
            r_true[e] = sqrt(gy * gy + gx * gx);
            theta_true[e] = o->f_atan2(gy, gx);
            scale_out[e] = sc;
        } else {
            r_true[e] = 0; theta_true[e] = 0; scale_out[e] = 0;
            o->flow_len[c] = 0;
            o->flow_theta[c] = 0;
        }
        o->last_time[c] = et; /* vFlow.cpp:407 */
    }
    return 0;
}
