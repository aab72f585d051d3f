// DecoderGPU::GetStats (the reference's batch boundary, QEC_LDPC/DecoderGPU.h:193-228) through the
// C++ interface: draws COUNT fixed-weight errors exactly as GetStatistics does (RandomErrorGenerator
// over mt19937(seed), QEC_LDPC/DecoderCPU.h:448-459), hands the flat COUNT x n arrays to GetStats,
// and prints both CodeStatistics' counters as one JSON line; they must be equal.  Optional
// --devices 0,0 runs GetStatistics on a multi-device decoder.
//   getstats_check CODEFILE W COUNT MAX P SEED [--devices LIST]
#include <cstdlib>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "DecoderGPU.h"
#include "RandomErrorGenerator.h"

static std::string counters(const CodeStatistics& s)
{
    std::ostringstream o;
    o << "[" << s.numErrorsTested << "," << s.numXErrorsTested << "," << s.numZErrorsTested << "," << s.corrected << ","
      << s.syndromeErrorsX << "," << s.syndromeErrorsZ << "," << s.logicalErrors << "," << s.convergenceFailX << ","
      << s.convergenceFailZ << "]";
    return o.str();
}

int main(int argc, char** argv)
{
    if (argc < 7) {
        std::cerr << "usage: getstats_check CODEFILE W COUNT MAX P SEED [--devices LIST]" << std::endl;
        return 2;
    }
    try {
        Quantum_LDPC_Code code = Quantum_LDPC_Code::createFromFile(argv[1]);
        const int W = std::atoi(argv[2]), COUNT = std::atoi(argv[3]), MAX = std::atoi(argv[4]);
        const float p = std::strtof(argv[5], nullptr);
        const unsigned seed = (unsigned)std::strtoul(argv[6], nullptr, 10);
        std::vector<int> devices{0};
        if (argc >= 9 && std::string(argv[7]) == "--devices") {
            devices.clear();
            std::stringstream ss(argv[8]);
            std::string tok;
            while (std::getline(ss, tok, ',')) devices.push_back(std::stoi(tok));
        }
        DecoderGPU one(code);
        RandomErrorGenerator gen(code.n, seed);
        std::vector<int> x((size_t)COUNT * code.n, 0), z((size_t)COUNT * code.n, 0);
        for (int s = 0; s < COUNT; ++s) {
            std::vector<int> ex(code.n, 0), ez(code.n, 0);
            gen.GenerateError(ex, ez, W);
            std::copy(ex.begin(), ex.end(), x.begin() + (size_t)s * code.n);
            std::copy(ez.begin(), ez.end(), z.begin() + (size_t)s * code.n);
        }
        const CodeStatistics a = one.GetStats(W, COUNT, p, MAX, (int)seed, x, z);
        DecoderGPU many(code, devices);
        const CodeStatistics b = many.GetStatistics(W, COUNT, p, MAX, seed);
        std::cout << "{\"getstats\": " << counters(a) << ", \"getstatistics\": " << counters(b)
                  << ", \"engine\": \"" << many.Describe() << "\"}" << std::endl;
        return counters(a) == counters(b) ? 0 : 1;
    } catch (const std::string& e) {
        std::cerr << e << std::endl;
        return 3;
    }
}
