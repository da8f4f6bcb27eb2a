// event_io.cpp — see event_io.h.
#include "event_io.h"

#include <climits>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>

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

int64_t parse_events(const char *text, size_t len, uint64_t max_events, EventColumns &cols) {
    // variables declared outside the loop, as vFlow.cpp:147
    int x = 0, y = 0, pol = 0;
    unsigned int t = 0;
    const char *p = text, *end = text + len;
    int64_t n = 0;
    while (p < end && (uint64_t)n < max_events) {  // getline && numEvents < NUMEVENTS
        const char *nl = (const char *)memchr(p, '\n', (size_t)(end - p));
        const char *le = nl ? nl : end;
        const char *q = p;
        bool fail = false;
        extract(q, le, x, fail);
        extract(q, le, y, fail);
        extract(q, le, t, fail);
        extract(q, le, pol, fail);
        cols.X.push_back(x);
        cols.Y.push_back(y);
        cols.T.push_back(t);
        cols.POL.push_back(pol);
        ++n;
        if (!nl) break;
        p = nl + 1;
    }
    return n;
}

bool read_events(const std::string &path, uint64_t max_events, EventColumns &cols, int64_t &n_read) {
    n_read = 0;
    std::ifstream f(path.c_str(), std::ios::binary);
    if (!f.is_open()) return false;
    std::string text((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    n_read = parse_events(text.data(), text.size(), max_events, cols);
    return true;
}

static size_t put_record(char *dst, const farms_records &r, int64_t i) {
    return (size_t)snprintf(dst, 256, "%d %d %d %d %g %g %g %g %g %g %d\n", r.x[i], r.y[i], r.t[i], r.p[i],
                            r.r_true[i], r.theta_true[i], r.vx[i], r.vy[i], r.r_local[i], r.theta_local[i],
                            r.scale[i]);
}

std::string format_records(const farms_records &r, int64_t begin, int64_t end) {
    std::string out;
    char line[256];
    for (int64_t i = begin; i < end; ++i) out.append(line, put_record(line, r, i));
    return out;
}

bool write_records(const std::string &path, const farms_records &r, int64_t n) {
    FILE *f = fopen(path.c_str(), "wb");
    if (!f) return false;
    std::vector<char> buf(1 << 22);
    size_t used = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (buf.size() - used < 256) { fwrite(buf.data(), 1, used, f); used = 0; }
        used += put_record(buf.data() + used, r, i);
    }
    fwrite(buf.data(), 1, used, f);
    return fclose(f) == 0;
}

}  // namespace farms_io

extern "C" int64_t farms_io_parse(const char *text, int64_t len, int64_t max_events, int32_t *x, int32_t *y,
                                  uint32_t *t, int32_t *p, int64_t cap) {
    farms_io::EventColumns cols;
    const int64_t n = farms_io::parse_events(text, (size_t)len, (uint64_t)max_events, cols);
    if (n > cap) return -1;
    for (int64_t i = 0; i < n; ++i) { x[i] = cols.X[i]; y[i] = cols.Y[i]; t[i] = cols.T[i]; p[i] = cols.POL[i]; }
    return n;
}

extern "C" int64_t farms_io_format(const farms_records *r, int64_t n, char *out, int64_t cap) {
    const std::string s = farms_io::format_records(*r, 0, n);
    if ((int64_t)s.size() + 1 > cap) return -1;
    memcpy(out, s.data(), s.size());
    out[s.size()] = '\0';
    return (int64_t)s.size();
}
