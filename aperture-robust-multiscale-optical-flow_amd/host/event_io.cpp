// event_io.cpp — see event_io.h.
#include "event_io.h"

#include <algorithm>
#include <charconv>
#include <climits>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <thread>

namespace farms_io {
namespace {

inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r'; }
inline bool is_digit(char c) { return c >= '0' && c <= '9'; }

// One `stream >> v` on an istringstream over [p, end), libstdc++ num_get rules:
// a stream already failed does nothing; skip white space; at the end of the
// line the sentry fails and v keeps its value; no digits -> v = 0; magnitude
// beyond the type -> v = its limit; either sets the fail state.  Unsigned
// targets accept a minus sign (modular negation), as strtoul does.
template <typename T>
void extract(const char *&p, const char *end, T &v, bool &fail) {
    if (fail) return;
    while (p < end && is_space(*p)) ++p;
    if (p == end) { fail = true; return; }
    bool neg = false;
    if (*p == '+' || *p == '-') { neg = *p == '-'; ++p; }
    if (p == end || !is_digit(*p)) { v = 0; fail = true; return; }
    const bool is_signed = T(-1) < T(0);
    const unsigned long long lim = is_signed ? (neg ? (unsigned long long)INT_MAX + 1ull : (unsigned long long)INT_MAX)
                                             : (unsigned long long)UINT_MAX;
    unsigned long long acc = 0;
    bool over = false;
    while (p < end && is_digit(*p)) {
        if (!over) {
            acc = acc * 10ull + (unsigned long long)(*p - '0');
            if (acc > lim) over = true;
        }
        ++p;
    }
    if (over) {
        if (is_signed) v = neg ? (T)INT_MIN : (T)INT_MAX;
        else v = (T)UINT_MAX;
        fail = true;
        return;
    }
    if (is_signed) v = neg ? (T)(0ll - (long long)acc) : (T)acc;
    else v = neg ? (T)(0u - (unsigned)acc) : (T)acc;
}

}  // namespace

namespace {

// Lines in [p, end): getline's count (a final line without '\n' counts).
int64_t count_lines(const char *p, const char *end) {
    int64_t n = 0;
    while (p < end) {
        const char *nl = (const char *)memchr(p, '\n', (size_t)(end - p));
        ++n;
        if (!nl) break;
        p = nl + 1;
    }
    return n;
}

// Parser state carried from line to line (vFlow.cpp:147 declares the four
// variables outside the loop). `known` tracks, per field, whether this chunk
// has assigned it yet; until then its lines carry the value the previous
// chunk ends with, which the fix-up pass fills in.
struct Carry {
    int x = 0, y = 0, pol = 0;
    unsigned int t = 0;
};

struct ChunkOut {
    int64_t first_def[4] = {-1, -1, -1, -1};  // first line (chunk-relative) that assigns field f
    Carry last;                               // values after the chunk's last line
};

// Parse `lines` lines of [p, end) into X/Y/T/P.
void parse_chunk(const char *p, const char *end, int64_t lines, int *X, int *Y, unsigned *T, int *P,
                 ChunkOut &co) {
    Carry c;
    for (int64_t i = 0; i < lines; ++i) {
        const char *nl = (const char *)memchr(p, '\n', (size_t)(end - p));
        const char *le = nl ? nl : end;
        const char *q = p;
        bool fail = false;
        // a field is assigned by extract() unless the stream has already failed
        // or the line ends before it; either way the variable keeps its value
        bool assigned[4];
        auto field = [&](int f, auto &v) {
            const char *w = q;
            while (w < le && is_space(*w)) ++w;
            assigned[f] = !fail && w < le;
            extract(q, le, v, fail);
        };
        field(0, c.x);
        field(1, c.y);
        field(2, c.t);
        field(3, c.pol);
        for (int f = 0; f < 4; ++f)
            if (assigned[f] && co.first_def[f] < 0) co.first_def[f] = i;
        X[i] = c.x; Y[i] = c.y; T[i] = c.t; P[i] = c.pol;
        if (!nl) break;
        p = nl + 1;
    }
    co.last = c;
}

}  // namespace

int64_t parse_events(const char *text, size_t len, uint64_t max_events, EventColumns &cols, int threads) {
    const char *end = text + len;
    // cap the text at max_events lines (getline && numEvents < NUMEVENTS)
    if (threads <= 0) {
        const unsigned hw = std::thread::hardware_concurrency();
        threads = (int)std::max(1u, std::min(hw ? hw : 1u, 16u));
        if (len < ((size_t)1 << 22)) threads = 1;  // small inputs: not worth the threads
    }
    // chunk boundaries at line starts
    std::vector<const char *> cut((size_t)threads + 1);
    cut[0] = text;
    for (int k = 1; k < threads; ++k) {
        const char *q = std::max(cut[(size_t)k - 1], text + len / (size_t)threads * (size_t)k);
        const char *nl = q < end ? (const char *)memchr(q, '\n', (size_t)(end - q)) : nullptr;
        cut[(size_t)k] = nl ? nl + 1 : end;
    }
    cut[(size_t)threads] = end;
    std::vector<int64_t> nl((size_t)threads), off((size_t)threads + 1, 0);
    auto run = [&](auto &&fn) {  // fn(k) for every chunk k; inline for chunks no thread could take
        std::vector<std::thread> pool;
        int k = 0;
        if (threads > 1) {
            try {
                for (; k < threads; ++k) pool.emplace_back(fn, k);
            } catch (...) {
            }
        }
        for (int j = k; j < threads; ++j) fn(j);
        for (auto &t : pool) t.join();
    };
    run([&](int k) { nl[(size_t)k] = count_lines(cut[(size_t)k], cut[(size_t)k + 1]); });
    for (int k = 0; k < threads; ++k) off[(size_t)k + 1] = off[(size_t)k] + nl[(size_t)k];
    const int64_t total = std::min<int64_t>(off[(size_t)threads], (int64_t)std::min<uint64_t>(max_events, INT64_MAX));
    const size_t base = cols.X.size();
    cols.X.resize(base + (size_t)total); cols.Y.resize(base + (size_t)total);
    cols.T.resize(base + (size_t)total); cols.POL.resize(base + (size_t)total);
    std::vector<ChunkOut> co((size_t)threads);
    run([&](int k) {
        const int64_t lo = std::min(off[(size_t)k], total), hi = std::min(off[(size_t)k + 1], total);
        if (hi > lo)
            parse_chunk(cut[(size_t)k], cut[(size_t)k + 1], hi - lo, cols.X.data() + base + lo,
                        cols.Y.data() + base + lo, cols.T.data() + base + lo, cols.POL.data() + base + lo,
                        co[(size_t)k]);
    });
    // fix-up, in chunk order: the leading lines of a chunk that carried a field
    // before assigning it take the value the previous chunk ended with
    Carry in;  // the reference's initial values (0)
    for (int k = 0; k < threads; ++k) {
        const int64_t lo = std::min(off[(size_t)k], total), hi = std::min(off[(size_t)k + 1], total);
        if (hi <= lo) continue;
        const int64_t len_k = hi - lo;
        const ChunkOut &o = co[(size_t)k];
        auto upto = [&](int f) { return o.first_def[f] < 0 ? len_k : o.first_def[f]; };
        for (int64_t i = 0; i < upto(0); ++i) cols.X[base + (size_t)(lo + i)] = in.x;
        for (int64_t i = 0; i < upto(1); ++i) cols.Y[base + (size_t)(lo + i)] = in.y;
        for (int64_t i = 0; i < upto(2); ++i) cols.T[base + (size_t)(lo + i)] = in.t;
        for (int64_t i = 0; i < upto(3); ++i) cols.POL[base + (size_t)(lo + i)] = in.pol;
        if (o.first_def[0] >= 0) in.x = o.last.x;
        if (o.first_def[1] >= 0) in.y = o.last.y;
        if (o.first_def[2] >= 0) in.t = o.last.t;
        if (o.first_def[3] >= 0) in.pol = o.last.pol;
    }
    return total;
}

bool read_events(const std::string &path, uint64_t max_events, EventColumns &cols, int64_t &n_read) {
    n_read = 0;
    std::string text;
    if (!read_text(path, text)) return false;
    n_read = parse_events(text.data(), text.size(), max_events, cols);
    return true;
}

bool read_text(const std::string &path, std::string &text) {
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) return false;
    char buf[1 << 16];
    if (fseek(f, 0, SEEK_END) == 0) {
        const long sz = ftell(f);
        if (sz > 0) text.reserve((size_t)sz);
        fseek(f, 0, SEEK_SET);
    }
    size_t got;
    while ((got = fread(buf, 1, sizeof(buf), f)) > 0) text.append(buf, got);
    fclose(f);
    return true;
}

int64_t parse_events_serial(const char *text, size_t len, uint64_t numevents, SerialEvents &out) {
    const char *p = text, *const end = text + len;
    int x = 0, y = 0, pol = 0;  // vFlow.cpp:494 (uninitialised there)
    unsigned int time_ = 0;
    auto line = [&](const char *&b, const char *&e) -> bool {  // getline
        if (p >= end) return false;
        const char *nl = (const char *)memchr(p, '\n', (size_t)(end - p));
        b = p;
        e = nl ? nl : end;
        p = nl ? nl + 1 : end;
        return true;
    };
    const char *b, *e;
    out.has_first = false;
    if (!line(b, e)) return 0;
    {  // the first line: only lastEventTime[x][y] = time_, t0 = time_ (vFlow.cpp:531-556)
        bool fail = false;
        extract(b, e, x, fail);
        extract(b, e, y, fail);
        extract(b, e, time_, fail);
        extract(b, e, pol, fail);
        out.has_first = true;
        out.x0 = x; out.y0 = y; out.t0 = time_;
    }
    const unsigned int t0 = time_;
    uint64_t computed = 0;  // eventsComputed (vFlow.cpp:76)
    while (line(b, e) && computed <= numevents) {  // vFlow.cpp:565
        bool fail = false;
        extract(b, e, x, fail);
        extract(b, e, y, fail);
        extract(b, e, time_, fail);
        time_ = time_ - t0;  // applied to a carried value too (vFlow.cpp:573)
        extract(b, e, pol, fail);
        if (pol < 0) pol = 0;  // vFlow.cpp:577-578
        out.cols.X.push_back(x);
        out.cols.Y.push_back(y);
        out.cols.T.push_back(time_);
        out.cols.POL.push_back(pol);
        ++computed;
    }
    return (int64_t)computed;
}

static size_t put_record(char *dst, const farms_records &r, int64_t i) {
    char *p = dst, *const end = dst + 256;
    const int32_t iv[4] = {r.x[i], r.y[i], r.t[i], r.p[i]};
    for (int k = 0; k < 4; ++k) {
        p = std::to_chars(p, end, iv[k]).ptr;
        *p++ = ' ';
    }
    const double dv[6] = {r.r_true[i], r.theta_true[i], r.vx[i], r.vy[i], r.r_local[i], r.theta_local[i]};
    for (int k = 0; k < 6; ++k) {
        p = std::to_chars(p, end, dv[k], std::chars_format::general, 6).ptr;
        *p++ = ' ';
    }
    p = std::to_chars(p, end, r.scale[i]).ptr;
    *p++ = '\n';
    return (size_t)(p - dst);
}

std::string format_records(const farms_records &r, int64_t begin, int64_t end) {
    std::string out;
    out.reserve((size_t)(end - begin) * 72);
    char line[256];
    for (int64_t i = begin; i < end; ++i) out.append(line, put_record(line, r, i));
    return out;
}

// Blocks of kBlock records are formatted by up to 16 threads at once, each
// into its own buffer, and written in order: the file is byte-identical to a
// sequential write, and host memory stays bounded (~16 x 8 MB).
bool write_records(const std::string &path, const farms_records &r, int64_t n) {
    FILE *f = fopen(path.c_str(), "wb");
    if (!f) return false;
    constexpr int64_t kBlock = 1 << 17;
    const unsigned hw = std::thread::hardware_concurrency();
    const int nt = (int)std::max(1u, std::min(hw ? hw : 1u, 16u));
    std::vector<std::string> bufs((size_t)nt);
    bool ok = true;
    for (int64_t b0 = 0; b0 < n && ok; b0 += kBlock * nt) {
        std::vector<std::thread> pool;
        int used = 0;
        for (int k = 0; k < nt; ++k) {
            const int64_t lo = b0 + k * kBlock, hi = std::min(n, lo + kBlock);
            if (lo >= hi) break;
            ++used;
            auto job = [&bufs, &r, k, lo, hi] { bufs[(size_t)k] = format_records(r, lo, hi); };
            bool spawned = false;
            if (nt > 1) {
                try {
                    pool.emplace_back(job);
                    spawned = true;
                } catch (...) {  // no thread available: format this block here
                }
            }
            if (!spawned) job();
        }
        for (auto &t : pool) t.join();
        for (int k = 0; k < used; ++k)
            ok = ok && fwrite(bufs[(size_t)k].data(), 1, bufs[(size_t)k].size(), f) == bufs[(size_t)k].size();
    }
    return fclose(f) == 0 && ok;
}

}  // namespace farms_io

extern "C" int64_t farms_io_parse_threads(const char *text, int64_t len, int64_t max_events, int32_t *x,
                                          int32_t *y, uint32_t *t, int32_t *p, int64_t cap, int threads) {
    farms_io::EventColumns cols;
    const int64_t n = farms_io::parse_events(text, (size_t)len, (uint64_t)max_events, cols, threads);
    if (n > cap) return -1;
    for (int64_t i = 0; i < n; ++i) { x[i] = cols.X[i]; y[i] = cols.Y[i]; t[i] = cols.T[i]; p[i] = cols.POL[i]; }
    return n;
}

extern "C" int64_t farms_io_parse(const char *text, int64_t len, int64_t max_events, int32_t *x, int32_t *y,
                                  uint32_t *t, int32_t *p, int64_t cap) {
    return farms_io_parse_threads(text, len, max_events, x, y, t, p, cap, 0);
}

extern "C" int64_t farms_io_format(const farms_records *r, int64_t n, char *out, int64_t cap) {
    const std::string s = farms_io::format_records(*r, 0, n);
    if ((int64_t)s.size() + 1 > cap) return -1;
    memcpy(out, s.data(), s.size());
    out[s.size()] = '\0';
    return (int64_t)s.size();
}

extern "C" int farms_io_write(const char *path, const farms_records *r, int64_t n) {
    return farms_io::write_records(path, *r, n) ? 0 : -1;
}

extern "C" int64_t farms_io_parse_serial(const char *text, int64_t len, int64_t numevents, int32_t *first3,
                                         int32_t *x, int32_t *y, uint32_t *t, int32_t *p, int64_t cap) {
    farms_io::SerialEvents se;
    const int64_t n = farms_io::parse_events_serial(text, (size_t)len, (uint64_t)numevents, se);
    if (n > cap) return -1;
    first3[0] = se.has_first ? 1 : 0;
    first3[1] = se.x0; first3[2] = se.y0; first3[3] = (int32_t)se.t0;
    for (int64_t i = 0; i < n; ++i) {
        x[i] = se.cols.X[(size_t)i]; y[i] = se.cols.Y[(size_t)i]; t[i] = se.cols.T[(size_t)i]; p[i] = se.cols.POL[(size_t)i];
    }
    return n;
}
