// main.cpp — FARMS_Flow command line, same flags and console output as the
// reference's Boost.program_options CLI (/root/reference/src/main.cpp:17-217).
//
//   FARMS_Flow --filename <file without .txt> --width W --height H
//              --filtersize F --inlierCheck K --numEvents N --SERIAL 0|1 --v 0|1
// Extensions: --windowJump J --maxWindow M (pooling scales, reference 5 / 50)
//             --device D (HIP device ordinal).
// Options accept "--name value" and "--name=value" and, like Boost's default
// style, any unambiguous prefix of a name.
#include <cmath>
#include <cstdlib>
#include <exception>
#include <iostream>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "vFlow.h"

namespace {

struct Opt {
    const char *name;
    bool takes_arg;
    const char *help;
};

const Opt kOpts[] = {
    {"help", false, "Displays this message"},
    {"filename", true, "add events file name without extension (.txt)"},
    {"height", true, "set sensor height"},
    {"width", true, "set sensor width"},
    {"filtersize", true, "set size of neighbor for plane fitting"},
    {"inlierCheck", true, "set minimum number of inliers to validate plane"},
    {"numEvents", true, "set max number of events to process"},
    {"numevents", true, "set max number of events to process"},
    {"NUMEVENTS", true, "set max number of events to process"},
    {"SERIAL", true, "Serial or Batch processing"},
    {"v", true, "set verbose to 1 for full debug mode"},
    {"windowJump", true, "[extension] pooling scale step (reference: 5)"},
    {"maxWindow", true, "[extension] largest pooling radius (reference: 50)"},
    {"device", true, "[extension] HIP device ordinal"},
};

void print_help() {
    std::cout << "Allowed options:\n";
    for (const Opt &o : kOpts) {
        std::string lhs = std::string("  --") + o.name + (o.takes_arg ? " arg" : "");
        if (lhs.size() < 24) lhs.resize(24, ' ');
        else lhs += " ";
        std::cout << lhs << o.help << "\n";
    }
}

const Opt *lookup(const std::string &name) {
    for (const Opt &o : kOpts)
        if (name == o.name) return &o;
    const Opt *hit = nullptr;  // unambiguous prefix (Boost allow_guessing)
    for (const Opt &o : kOpts)
        if (std::string(o.name).compare(0, name.size(), name) == 0) {
            if (hit) throw std::runtime_error("option '--" + name + "' is ambiguous");
            hit = &o;
        }
    if (!hit) throw std::runtime_error("unrecognised option '--" + name + "'");
    return hit;
}

int as_int(const std::map<std::string, std::string> &vm, const char *name) {
    const std::string &v = vm.at(name);
    size_t used = 0;
    long long r = 0;
    try {
        r = std::stoll(v, &used);
    } catch (...) {
        used = 0;
    }
    if (used != v.size() || r < INT32_MIN || r > INT32_MAX)
        throw std::runtime_error("the argument ('" + v + "') for option '--" + name + "' is invalid");
    return (int)r;
}

}  // namespace

int main(int argc, char *argv[]) {
    // defaults of main.cpp:21-31
    int height = 320, width = 320, filterSize = 3, minEvtsOnPlane = 5;
    int windowJump = 5, maxWindow = 50, device = 0;
    bool verboseMode = false;
    unsigned long int NUMEVENTS = (unsigned long int)std::pow(2, 63);
    std::string fileNameInput = "events";
    bool Serial_ = true;
    try {
        std::map<std::string, std::string> vm;
        for (int i = 1; i < argc; ++i) {
            std::string a = argv[i];
            if (a.size() < 3 || a[0] != '-' || a[1] != '-') throw std::runtime_error("unrecognised option '" + a + "'");
            a = a.substr(2);
            std::string val;
            bool has_val = false;
            const size_t eq = a.find('=');
            if (eq != std::string::npos) { val = a.substr(eq + 1); a = a.substr(0, eq); has_val = true; }
            const Opt *o = lookup(a);
            if (o->takes_arg && !has_val) {
                if (i + 1 >= argc) throw std::runtime_error(std::string("the required argument for option '--") + o->name + "' is missing");
                val = argv[++i];
            }
            if (vm.count(o->name)) throw std::runtime_error(std::string("option '--") + o->name + "' cannot be specified more than once");
            vm[o->name] = val;
        }
        if (vm.count("help")) {
            print_help();
            return 0;
        }
        if (vm.count("v")) {
            std::cout << "Verbose mode set to " << as_int(vm, "v") << std::endl;
            if (as_int(vm, "v") == 1) verboseMode = true;
        }
        if (vm.count("filename")) {
            std::cout << "filename set to " << vm["filename"] << ".\n";
            fileNameInput = vm["filename"];
        }
        if (vm.count("height")) { height = as_int(vm, "height"); std::cout << "height set to " << height << ".\n"; }
        if (vm.count("width")) { width = as_int(vm, "width"); std::cout << "width set to " << width << ".\n"; }
        if (vm.count("filtersize")) {
            filterSize = as_int(vm, "filtersize");
            std::cout << "filtersize set to " << filterSize << ".\n";
        }
        if (vm.count("inlierCheck")) {
            minEvtsOnPlane = as_int(vm, "inlierCheck");
            std::cout << "inlierCheck set to " << minEvtsOnPlane << ".\n";
        }
        for (const char *k : {"numEvents", "numevents", "NUMEVENTS"})  // first one given wins (main.cpp:131-151)
            if (vm.count(k)) {
                const int v = as_int(vm, k);
                std::cout << "numEvents set to " << v << ".\n";
                NUMEVENTS = (unsigned long int)(long)v;
                break;
            }
        if (vm.count("SERIAL")) {
            if (as_int(vm, "SERIAL") == 1) { std::cout << "Running serially " << std::endl; Serial_ = true; }
            else { Serial_ = false; std::cout << "Running batch " << std::endl; }
        }
        if (vm.count("windowJump")) windowJump = as_int(vm, "windowJump");
        if (vm.count("maxWindow")) maxWindow = as_int(vm, "maxWindow");
        if (vm.count("device")) device = as_int(vm, "device");
    } catch (std::exception &e) {
        std::cerr << "error: " << e.what() << "\n";
        return 1;
    }

    try {
        vFlowManager vFlowM(height, width, filterSize, minEvtsOnPlane, fileNameInput);
        vFlowM.setScales(windowJump, maxWindow);
        vFlowM.setDevice(device);
        std::cout << "[debug Main] : size of lastFlowTime is [sx sy]: [" << vFlowM.returnFlowTime().dim_a() << " "
                  << vFlowM.returnFlowTime().dim_b() << "]" << std::endl;
        vFlowM.setDebugMode(verboseMode);
        const long durationActualProcessing = Serial_ ? vFlowM.run(NUMEVENTS) : vFlowM.runFileCopy(NUMEVENTS);
        // main.cpp:200-201 / 208-209, including the integer-second truncation
        float durationActualProcessingSec = durationActualProcessing / 1000000;
        std::cout << "[Benchmark Main] : Processing time   : " << durationActualProcessing << " usec "
                  << durationActualProcessingSec << " sec "
                  << " with rate of : " << (vFlowM.getNumEvents() - 1) / durationActualProcessingSec << " events/sec"
                  << std::endl;
        // exact rate (the line above keeps the reference's truncation)
        std::cout << "[Benchmark Main] : " << vFlowM.getNumEvents() / (durationActualProcessing * 1e-6)
                  << " events/sec (microsecond timer)" << std::endl;
    } catch (std::exception &e) {
        std::cerr << "error: " << e.what() << "\n";
        return 2;
    }
    return 0;
}
