// vFlow.h — host-side vFlowManager over the MI355X C ABI.
//
// Same public interface as the reference class (/root/reference/include/vFlow.h:
// 22-117) so that main.cpp-style callers drop in unchanged: the constructor
// takes (height, width, filterSize, minEvtsOnPlane, fileName), runFileCopy(N)
// reads <fileName>.txt, runs the per-event loop and writes
// <fileName>_FARMSOut_batch.txt, returning the microseconds of the timed loop
// (vFlow.cpp:111-460).  The per-event loop itself runs on the GPU through
// libfarms_hip.so (include/farms_hip.h); parsing, t0 subtraction, polarity
// clamping, timing and the writer stay here, as in the reference.
#ifndef FARMS_HOST_VFLOW_H
#define FARMS_HOST_VFLOW_H

#include <string>
#include <vector>

#include "Event.h"
#include "FlowEvent.h"
#include "farms_hip.h"

// Minimal W x H grid with the reference's x-major indexing (EventMatrix.h:32-37):
// m[x][y] is element x*dim_b() + y.
template <class T>
class EventMatrix {
public:
    EventMatrix() : b_(0) {}
    EventMatrix(int a, int b, const T &init = T()) : data_((size_t)a * b, init), b_(b) {}
    int dim_a() const { return b_ ? (int)(data_.size() / b_) : 0; }
    int dim_b() const { return b_; }
    T *operator[](int a) { return &data_[(size_t)a * b_]; }
    const T *operator[](int a) const { return &data_[(size_t)a * b_]; }
    T *data() { return data_.data(); }

private:
    std::vector<T> data_;
    int b_;
};

class vFlowManager {
public:
    vFlowManager(int height, int width, int filterSize, int minEvtsOnPlane);
    vFlowManager(int height, int width, int filterSize, int minEvtsOnPlane, std::string fileName);
    ~vFlowManager();
    vFlowManager(const vFlowManager &) = delete;
    vFlowManager &operator=(const vFlowManager &) = delete;

    long run(unsigned long int NUMEVENTS);          // serial mode, see vFlow.cpp
    long runFileCopy(unsigned long int NUMEVENTS);  // batch mode -> _FARMSOut_batch.txt
    void close();

    EventMatrix<double> returnFlowTime();  // lastEventTime surface (x-major)
    double getNumEvents() { return numEvents; }
    void setDebugMode(bool in) { DEBUGMODE = in; }

    // extensions (not in the reference): pooling scales and placement
    void setScales(int windowJump, int maxWindow);
    void setDevice(int device);

    std::vector<int> X;
    std::vector<int> Y;
    std::vector<unsigned int> T;
    std::vector<int> POL;

private:
    long process(bool write_output);
    int ensure_handle();
    void print_serial_timing(long us, const double *vx, const double *vy, int64_t n);

    bool DEBUGMODE = false;
    double numEvents = 0;
    std::string fileNameInput;
    farms_params prm{};
    farms_handle *handle = nullptr;
};

#endif
