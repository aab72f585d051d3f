// qec_ldpc -- the reference's Monte-Carlo driver (QEC_LDPC/main.cu:43-118) on the
// MI355X engine.  Same init-file format ("codeFile w W COUNT MAX p", main.cu:74-88),
// same results files (results/<code>_W_<w>_MAX_<MAX>_p_<p>.txt, appended,
// main.cu:91-104) and the same output_log.txt journal (main.cu:45-52,114).
// The only change vs main.cu is the engine: DecoderGPU instead of DecoderCPU.
// Exit status is 0 on success (main.cu returns 1).
// Optional flags before the init file ("Config / flags"):
//   --engine gpu|cpu   the decoder: DecoderGPU (default) or DecoderCPU (host threads, no GPU needed)
//   --gpus N           GPUs 0..N-1 of this node, one decoder spanning them (counters identical to one GPU)
//   --devices 0,3,5    the same for a list of GPUs
//   --rng msvc|philox  msvc (default): main.cu's loop, fixed-weight errors w..W from the reference's
//                      mt19937 stream (GetStatistics, reference stop rule).  philox: COUNT i.i.d.
//                      depolarising samples at p per run (qec_monte_carlo, GPU engine), w and W ignored
//   --stop ref|fixed|syndrome   stop rule of --rng philox runs (default ref)
//   --batch B          samples per device batch of --rng philox runs (default 2^20)
//   --seed S           Philox stream of --rng philox runs (default 0x51EC0DE; GetStatistics draws its
//                      own seed from std::random_device, as main.cu does)
// Unknown or inconsistent flags exit with status 2.
#include <algorithm>
#include <chrono>
#include <ctime>
#include <fstream>
#include <iostream>
#include <memory>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "DecoderCPU.h"
#include "DecoderGPU.h"
#include "Quantum_LDPC_Code.h"

namespace {

// One --rng philox run's block in the results file (the CodeStatistics fields that exist for
// depolarising samples, plus the stop rule and the iterations executed)
void write_mc_block(std::ostream& out, const Quantum_LDPC_Code& code, unsigned long long seed, float p, int maxIter,
                    const char* stop, const qec_mc_result& r)
{
    out << "Code: " << code << std::endl
        << "Philox Seed: " << seed << std::endl
        << "Duration(micro-s): " << (long long)(r.totalSeconds * 1e6) << std::endl
        << "Physical Error Rate: " << p << std::endl
        << "Stop Rule: " << stop << std::endl
        << "Max Iterations: " << maxIter << std::endl
        << "Errors Tested: " << r.tested << std::endl
        << "Errors With X: " << r.withX << std::endl
        << "Errors With Z: " << r.withZ << std::endl
        << "Corrected: " << r.corrected << std::endl
        << "Syndrome Errors X: " << r.synX << std::endl
        << "Syndrome Errors Z: " << r.synZ << std::endl
        << "Logical Errors: " << r.logical << std::endl
        << "Convergence Fail X: " << r.convX << std::endl
        << "Convergence Fail Z: " << r.convZ << std::endl
        << "Iterations X: " << r.iterationsX << std::endl
        << "Iterations Z: " << r.iterationsZ << std::endl;
}

int usage(const std::string& why)
{
    std::cerr << why << std::endl
              << "usage: qec_ldpc [--engine gpu|cpu] [--gpus N | --devices i,j,...] [--rng msvc|philox]"
                 " [--stop ref|fixed|syndrome] [--batch B] [--seed S] initFile"
              << std::endl;
    return 2;
}

}  // namespace

int main(int argc, char** argv)
{
    std::ofstream log("output_log.txt", std::ios::app);
    if (!log.is_open()) {
        std::cerr << "Unable to open output log file" << std::endl;
        return 2;
    }
    std::time_t ts = std::chrono::system_clock::to_time_t(std::chrono::system_clock::now());
    log << std::endl << std::ctime(&ts);
    std::vector<int> devices{0};
    std::string engine = "gpu", rng = "msvc", stopName = "ref";
    bool deviceFlag = false, stopFlag = false, batchFlag = false, seedFlag = false;
    size_t batch = size_t(1) << 20;
    unsigned long long seed = 0x51EC0DE;
    int a = 1;
    try {
        for (; a + 1 < argc && std::string(argv[a]).rfind("--", 0) == 0; a += 2) {
            const std::string flag = argv[a], val = argv[a + 1];
            if (flag == "--gpus" || flag == "--devices") {
                devices.clear();
                deviceFlag = true;
                if (flag == "--gpus") {
                    for (int k = 0; k < std::stoi(val); ++k) devices.push_back(k);
                } else {
                    std::stringstream ss(val);
                    std::string tok;
                    while (std::getline(ss, tok, ',')) devices.push_back(std::stoi(tok));
                }
            } else if (flag == "--engine") {
                engine = val;
                if (engine != "gpu" && engine != "cpu") return usage("--engine: gpu or cpu");
            } else if (flag == "--rng") {
                rng = val;
                if (rng != "msvc" && rng != "philox") return usage("--rng: msvc or philox");
            } else if (flag == "--stop") {
                stopName = val;
                stopFlag = true;
                if (stopName != "ref" && stopName != "fixed" && stopName != "syndrome")
                    return usage("--stop: ref, fixed or syndrome");
            } else if (flag == "--batch") {
                const long long b = std::stoll(val);
                if (b <= 0) return usage("--batch: a positive sample count");
                batch = (size_t)b;
                batchFlag = true;
            } else if (flag == "--seed") {
                seed = std::stoull(val, nullptr, 0);
                seedFlag = true;
            } else {
                return usage("unknown flag " + flag);
            }
        }
    } catch (const std::exception&) {
        return usage("unreadable flag value");
    }
    if (engine == "cpu" && deviceFlag) return usage("--gpus / --devices need --engine gpu");
    if (rng == "philox" && engine == "cpu") return usage("--rng philox runs on the GPU engine only");
    if (rng == "msvc" && (stopFlag || batchFlag || seedFlag))
        return usage("--stop / --batch / --seed apply to --rng philox (GetStatistics keeps the reference stop rule)");
    if (argc - a != 1 || devices.empty()) {
        log << "Must provide initialization file." << std::endl;
        return 0;
    }
    std::string initFile = argv[a];
    std::ifstream init(initFile);
    if (!init.is_open()) {
        log << "Unable to open init file \"" << initFile
            << "\". Please make sure the file exists in the current directory." << std::endl;
        return 0;
    }
    log << "Initializing run from file " << initFile << std::endl;
    std::string codeFile;
    init >> codeFile;
    try {
        std::cout << "Creating code from file " << codeFile << std::endl;
        Quantum_LDPC_Code code = Quantum_LDPC_Code::createFromFile(codeFile);
        int w, W, COUNT, MAX_ITERATIONS;
        float p;
        init >> w >> W >> COUNT >> MAX_ITERATIONS >> p;
        const bool read_ok = !init.fail();
        init.close();
        if (!read_ok || COUNT < 0 || MAX_ITERATIONS < 0) {
            // main.cu:74-88 reads the same fields; a negative or unread COUNT would wrap to ~1.8e19 samples
            // in the Philox run below (main.cu's own loop just does nothing then)
            std::cerr << initFile << ": expected 'codeFile w W COUNT MAX p' with COUNT >= 0 and MAX >= 0" << std::endl;
            return 2;
        }
        if (rng == "philox") {
            DecoderGPU decoder(code, devices);
            std::cout << "Engine: " << decoder.Describe() << std::endl;
            const int stop = stopName == "ref" ? QEC_STOP_REF : stopName == "fixed" ? QEC_STOP_FIXED : QEC_STOP_SYNDROME;
            std::stringstream fileName;
            fileName << "results/" << code << "_DEPOLARIZING_MAX_" << MAX_ITERATIONS << "_p_" << p << "_" << stopName
                     << ".txt";
            std::string str = fileName.str();
            str.erase(std::remove(str.begin(), str.end(), ' '), str.end());
            std::cout << str << std::endl;
            std::ofstream outFile(str, std::ios_base::app);
            qec_mc_result r{};
            if (qec_monte_carlo(decoder.handle(), seed, 0, (uint64_t)COUNT, p, MAX_ITERATIONS, stop, batch, &r) != QEC_OK)
                throw std::string(qec_last_error());
            write_mc_block(outFile, code, seed, p, MAX_ITERATIONS, stopName.c_str(), r);
            outFile << std::endl;
            log << "Run complete." << std::endl;
            return 0;
        }
        std::unique_ptr<Decoder> decoder;
        if (engine == "cpu") {
            decoder.reset(new DecoderCPU(code));
            std::cout << "Engine: CPU (" << std::thread::hardware_concurrency() << " threads)" << std::endl;
        } else {
            DecoderGPU* g = new DecoderGPU(code, devices);
            decoder.reset(g);
            std::cout << "Engine: " << g->Describe() << std::endl;
        }
        for (; w <= W; ++w) {
            std::stringstream fileName;
            fileName << "results/" << code << "_W_" << w << "_MAX_" << MAX_ITERATIONS << "_p_" << p << ".txt";
            std::string str = fileName.str();
            str.erase(std::remove(str.begin(), str.end(), ' '), str.end());
            std::cout << str << std::endl;
            std::ofstream outFile(str, std::ios_base::app);
            CodeStatistics stats = decoder->GetStatistics(w, COUNT, p, MAX_ITERATIONS);
            outFile << stats << std::endl << std::endl;
        }
    } catch (const std::string& s) {
        log << s << std::endl;
        std::cerr << s << std::endl;
        return 1;
    }
    log << "Run complete." << std::endl;
    return 0;
}
