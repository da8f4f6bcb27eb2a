// event_io.h — the text formats of the FARMS_Flow batch path.
//
// Input: one "x y t p" line per event (/root/reference/README.md, "Input event
// files"), read with the exact semantics of the reference's parser
// (src/vFlow.cpp:147,173-188): getline + four `stream >> v` extractions into
// variables that live across lines, so a short or malformed line repeats the
// previous values for the fields it cannot supply; a field that fails to
// convert becomes 0 (an out-of-range one saturates) and the rest of its line
// is skipped.
// Output: the 11 columns of src/vFlow.cpp:438 with std::ostream defaults
// (integers, doubles as %.6g), one line per event.
#ifndef FARMS_HOST_EVENT_IO_H
#define FARMS_HOST_EVENT_IO_H

#include <cstdint>
#include <string>
#include <vector>

#include "farms_hip.h"

namespace farms_io {

struct EventColumns {
    std::vector<int> X, Y, POL;
    std::vector<unsigned int> T;
};

// Parse the events of `text` (a whole file) into cols, at most max_events
// lines.  Returns the number of events appended.  Chunks of lines are parsed
// on `threads` threads (0: up to 16, one for inputs under 4 MB); the values a
// chunk's leading lines carry over from the previous line are filled in
// afterwards, so the result equals the one-thread parse.
int64_t parse_events(const char *text, size_t len, uint64_t max_events, EventColumns &cols, int threads = 0);

// Read and parse a file.  Returns false if it cannot be opened.
bool read_events(const std::string &path, uint64_t max_events, EventColumns &cols, int64_t &n_read);

// Read a whole file.  Returns false if it cannot be opened.
bool read_text(const std::string &path, std::string &text);

// vFlowManager::run's reading (vFlow.cpp:520-580), one thread: the first line
// gives (x0, y0, t0) and is not an event; then lines while eventsComputed <=
// numevents (at most numevents + 1 events), parsed into the same variables
// with `time_ = time_ - t0` after each time extraction (so a line without a
// time field subtracts t0 once more from the carried relative stamp) and the
// polarity clamped to >= 0 in place.  cols.T holds relative stamps, cols.POL
// clamped polarities.  Returns the number of events.
struct SerialEvents {
    bool has_first = false;
    int x0 = 0, y0 = 0;
    unsigned int t0 = 0;
    EventColumns cols;
};
int64_t parse_events_serial(const char *text, size_t len, uint64_t numevents, SerialEvents &out);

// Format n records (host arrays) as the _FARMSOut_ text.
std::string format_records(const farms_records &r, int64_t begin, int64_t end);
bool write_records(const std::string &path, const farms_records &r, int64_t n);

}  // namespace farms_io

// C ABI used by the CPU tests (tests/test_host_io.py)
extern "C" {
int64_t farms_io_parse(const char *text, int64_t len, int64_t max_events, int32_t *x, int32_t *y,
                       uint32_t *t, int32_t *p, int64_t cap);
int64_t farms_io_format(const farms_records *r, int64_t n, char *out, int64_t cap);
// first3 = {has_first, x0, y0, t0}
int64_t farms_io_parse_serial(const char *text, int64_t len, int64_t numevents, int32_t *first3, int32_t *x,
                              int32_t *y, uint32_t *t, int32_t *p, int64_t cap);
}

#endif
