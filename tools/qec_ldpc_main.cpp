// qec_ldpc -- the reference's Monte-Carlo driver (QEC_LDPC/main.cu:43-118) on the
// MI355X engine.  Same init-file format ("codeFile w W COUNT MAX p", main.cu:74-88),
// same results files (results/<code>_W_<w>_MAX_<MAX>_p_<p>.txt, appended,
// main.cu:91-104) and the same output_log.txt journal (main.cu:45-52,114).
// The only change vs main.cu is the engine: DecoderGPU instead of DecoderCPU.
// Exit status is 0 on success (main.cu returns 1).
// Optional flags before the init file: --gpus N (GPUs 0..N-1 of this node, one decoder
// spanning them; counters are identical to one GPU) or --devices 0,3,5.
#include <algorithm>
#include <chrono>
#include <ctime>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "DecoderGPU.h"
#include "Quantum_LDPC_Code.h"

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
    int a = 1;
    for (; a + 1 < argc && std::string(argv[a]).rfind("--", 0) == 0; a += 2) {
        const std::string flag = argv[a], val = argv[a + 1];
        devices.clear();
        if (flag == "--gpus") {
            for (int k = 0; k < std::stoi(val); ++k) devices.push_back(k);
        } else if (flag == "--devices") {
            std::stringstream ss(val);
            std::string tok;
            while (std::getline(ss, tok, ',')) devices.push_back(std::stoi(tok));
        } else {
            std::cerr << "unknown flag " << flag << std::endl;
            return 2;
        }
    }
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
        DecoderGPU decoder(code, devices);
        std::cout << "Engine: " << decoder.Describe() << std::endl;
        int w, W, COUNT, MAX_ITERATIONS;
        float p;
        init >> w >> W >> COUNT >> MAX_ITERATIONS >> p;
        init.close();
        for (; w <= W; ++w) {
            std::stringstream fileName;
            fileName << "results/" << code << "_W_" << w << "_MAX_" << MAX_ITERATIONS << "_p_" << p << ".txt";
            std::string str = fileName.str();
            str.erase(std::remove(str.begin(), str.end(), ' '), str.end());
            std::cout << str << std::endl;
            std::ofstream outFile(str, std::ios_base::app);
            CodeStatistics stats = decoder.GetStatistics(w, COUNT, p, MAX_ITERATIONS);
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
