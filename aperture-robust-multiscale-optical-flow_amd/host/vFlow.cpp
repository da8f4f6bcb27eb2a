// vFlow.cpp — host-side vFlowManager (see vFlow.h).
//
// runFileCopy follows /root/reference/src/vFlow.cpp:111-460 step for step:
// same console lines, same file names, same parse semantics (event_io), same
// timed region (after the parse, before the write), same 11 output columns.
// The per-event loop (vFlow.cpp:223-414) is one farms_process call.
#include "vFlow.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <string>
#include <cstdlib>
#include <iostream>
#include <stdexcept>

#include "event_io.h"

namespace {
// An array in pinned host memory (farms_host_alloc): farms_process DMAs it in
// place instead of staging it.
template <class T>
struct Pinned {
    T *ptr = nullptr;
    explicit Pinned(size_t n) {
        void *v = nullptr;
        if (farms_host_alloc((int64_t)(n * sizeof(T)), &v) != FARMS_OK)
            throw std::runtime_error(std::string("farms_host_alloc: ") + farms_last_error());
        ptr = static_cast<T *>(v);
    }
    ~Pinned() { farms_host_free(ptr); }
    Pinned(const Pinned &) = delete;
    Pinned &operator=(const Pinned &) = delete;
    T &operator[](size_t i) { return ptr[i]; }
};
}  // namespace

vFlowManager::vFlowManager(int height, int width, int filterSize, int minEvtsOnPlane)
    : vFlowManager(height, width, filterSize, minEvtsOnPlane, std::string()) {}

vFlowManager::vFlowManager(int height, int width, int filterSize, int minEvtsOnPlane, std::string fileName) {
    std::cout << "[debug] : Begin creating vFlowManager object" << std::endl;  // vFlow.cpp:26
    farms_default_params(&prm);
    prm.height = height;
    prm.width = width;
    prm.filter_size = filterSize;  // normalised by the library as vFlow.cpp:32-36
    prm.min_inliers = minEvtsOnPlane;
    fileNameInput = fileName;
}

vFlowManager::~vFlowManager() { close(); }

void vFlowManager::close() {
    if (handle) farms_destroy(handle);
    handle = nullptr;
}

void vFlowManager::setScales(int windowJump, int maxWindow) {
    prm.window_jump = windowJump;
    prm.max_window = maxWindow;
    close();
}

void vFlowManager::setDevice(int device) {
    prm.device = device;
    close();
}

int vFlowManager::ensure_handle() {
    if (handle) return FARMS_OK;
    return farms_create(&prm, &handle);
}

EventMatrix<double> vFlowManager::returnFlowTime() {
    EventMatrix<double> m(prm.width, prm.height, 0.0);
    if (handle) farms_get_last_event_time(handle, m.data());
    return m;
}

// The timed per-event loop over the parsed X/Y/T/POL (vFlow.cpp:194-423).
long vFlowManager::process(bool write_output) {
    const int64_t n = (int64_t)T.size();
    if (n == 0) {
        // the reference dies here with std::out_of_range from T.at(0) (vFlow.cpp:194)
        throw std::out_of_range("no events read from " + fileNameInput);
    }
    const unsigned int t0 = T.at(0);
    std::cout << "First time = " << t0 << std::endl;
    std::cout << "Processing events " << std::endl;
    if (prm.serial) {  // runFileCopy after run(): batch semantics again
        prm.serial = 0;
        close();
    }
    int rc = ensure_handle();
    if (rc != FARMS_OK) throw std::runtime_error(std::string("farms_create: ") + farms_last_error());

    // the loop's own arrays in pinned memory: DMAed in place (X and Y, the
    // reference's public vectors, go through the library's staging)
    const size_t un = (size_t)n;
    Pinned<uint32_t> t_rel(un);
    Pinned<int32_t> p(un), ox(un), oy(un), ot(un), op(un), osc(un);
    Pinned<double> rt(un), tt(un), vx(un), vy(un), rl(un), tl(un);
    farms_records rec{ox.ptr, oy.ptr, ot.ptr, op.ptr, rt.ptr, tt.ptr, vx.ptr, vy.ptr, rl.ptr, tl.ptr, osc.ptr};

    const auto start = std::chrono::system_clock::now();  // vFlow.cpp:214
    for (int64_t e = 0; e < n; ++e) {
        t_rel[(size_t)e] = T[(size_t)e] - t0;                   // vFlow.cpp:240-241
        p[(size_t)e] = POL[(size_t)e] < 0 ? 0 : POL[(size_t)e];  // vFlow.cpp:245-247
    }
    rc = farms_process(handle, X.data(), Y.data(), t_rel.ptr, p.ptr, n, &rec);
    const auto stop = std::chrono::system_clock::now();  // vFlow.cpp:416
    if (rc != FARMS_OK) throw std::runtime_error(std::string("farms_process: ") + farms_last_error());
    numEvents += (double)n;
    const long us = (long)std::chrono::duration_cast<std::chrono::microseconds>(stop - start).count();

    std::cout << std::endl << "Done processing!" << std::endl;
    if (write_output) {
        std::cout << std::endl << "Writing output file." << std::endl;
        const std::string out = fileNameInput + "_FARMSOut_batch.txt";  // vFlow.cpp:131
        if (!farms_io::write_records(out, rec, n)) std::cerr << "cannot write " << out << std::endl;
    }
    return us;
}

long vFlowManager::runFileCopy(unsigned long int NUMEVENTS) {
    const std::string in = fileNameInput + ".txt";  // vFlow.cpp:150
    std::cout << in << std::endl;
    std::cout << "Reading input file " << std::endl;
    farms_io::EventColumns cols;
    int64_t nread = 0;
    farms_io::read_events(in, NUMEVENTS, cols, nread);  // an unopenable file reads 0 events
    X.insert(X.end(), cols.X.begin(), cols.X.end());
    Y.insert(Y.end(), cols.Y.begin(), cols.Y.end());
    T.insert(T.end(), cols.T.begin(), cols.T.end());
    POL.insert(POL.end(), cols.POL.begin(), cols.POL.end());
    std::cout << "Done reading " << nread << " Events." << std::endl;
    return process(true);
}

// Serial mode (vFlow.cpp:465-826), the reference CLI's default: the first
// line only stamps lastEventTime (farms_serial_first), the loop runs over at
// most NUMEVENTS + 1 further lines with the engine's serial semantics
// (lastEventTime written after pooling, farms_params.serial) and writes no
// output; returns the microseconds of the accelerated loop.  The reference
// prints a "Local <us> <cumulative us>" line per event and a "true <us>
// <cumulative us>" line per valid one (vFlow.cpp:641, 719): host timings of
// each event's two phases.  Here the loop is one batched device call, so no
// event has a duration of its own; instead of per-event lines that would look
// like measurements, one line reports what was measured: the whole call.
void vFlowManager::print_serial_timing(long us, const double *vx, const double *vy, int64_t n) {
    int64_t nvalid = 0;
    for (int64_t e = 0; e < n; ++e)  // the validity gate of vFlow.cpp:645
        nvalid += !std::isnan(vx[e]) && !std::isnan(vy[e]) && vx[e] != 0 && vy[e] != 0;
    std::cout << "Batch " << n << " events " << nvalid << " valid " << us
              << " us (one device call: no per-event Local / true timings)" << std::endl;
}

long vFlowManager::run(unsigned long int NUMEVENTS) {
    const std::string in = fileNameInput + ".txt";  // vFlow.cpp:497
    std::cout << in << std::endl;
    std::string text;
    if (!farms_io::read_text(in, text)) {
        std::cout << "Unable to open file" << std::endl;  // vFlow.cpp:802
        std::cout << std::endl << "Done!" << std::endl;
        return 0;
    }
    // NUMEVENTS = min(NUMEVENTS, fsize / 18) (vFlow.cpp:513)
    NUMEVENTS = (unsigned long int)std::min<double>((double)NUMEVENTS, (double)(text.size() / 18));
    farms_io::SerialEvents se;
    const int64_t n = farms_io::parse_events_serial(text.data(), text.size(), NUMEVENTS, se);
    std::string().swap(text);
    if (!se.has_first) {
        std::cout << std::endl << "Done!" << std::endl;
        return 0;
    }
    std::cout << "First time = " << se.t0 << std::endl;  // vFlow.cpp:549
    if (!prm.serial) {
        prm.serial = 1;
        close();
    }
    int rc = ensure_handle();
    if (rc != FARMS_OK) throw std::runtime_error(std::string("farms_create: ") + farms_last_error());
    rc = farms_serial_first(handle, se.x0, se.y0, se.t0);
    if (rc != FARMS_OK) throw std::runtime_error(std::string("farms_serial_first: ") + farms_last_error());
    long us = 0;
    if (n > 0) {
        std::vector<int32_t> ox((size_t)n), oy((size_t)n), ot((size_t)n), op((size_t)n), osc((size_t)n);
        std::vector<double> rt((size_t)n), tt((size_t)n), vx((size_t)n), vy((size_t)n), rl((size_t)n), tl((size_t)n);
        farms_records rec{ox.data(), oy.data(), ot.data(), op.data(), rt.data(), tt.data(),
                          vx.data(), vy.data(), rl.data(), tl.data(), osc.data()};
        const auto start = std::chrono::system_clock::now();
        rc = farms_process(handle, se.cols.X.data(), se.cols.Y.data(), se.cols.T.data(), se.cols.POL.data(), n, &rec);
        const auto stop = std::chrono::system_clock::now();
        if (rc != FARMS_OK) throw std::runtime_error(std::string("farms_process: ") + farms_last_error());
        us = (long)std::chrono::duration_cast<std::chrono::microseconds>(stop - start).count();
        numEvents += (double)n;  // this->numEvents = eventsComputed (vFlow.cpp:792)
        print_serial_timing(us, vx.data(), vy.data(), n);
    }
    std::cout << std::endl << "Done!" << std::endl;  // vFlow.cpp:808
    return us;
}
