// DecoderCPU.h -- the reference's CPU decoder class (QEC_LDPC/DecoderCPU.h:16-530), backed by the
// CPU engine of libqecldpc.so (qec_decoder_create with device -1): host threads over edge-major
// tables, the reference's arithmetic operation for operation, so decisions, flags and
// CodeStatistics counters are bit-identical.  Same class name and signatures, so the unmodified
// `DecoderCPU decoder(code);` of QEC_LDPC/main.cu:79 builds against this repository.
//
// Decode takes the base class's std::vector arguments, so it overrides Decoder::Decode (the
// reference's cusp vectors hid it instead).
#pragma once
#include <cstdint>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "Decoder.h"

class DecoderCPU : public Decoder {
public:
    explicit DecoderCPU(Quantum_LDPC_Code code) : Decoder(code)
    {
        dec_ = qec_decoder_create(_code.handle(), -1, 0);
        if (!dec_) throw std::string(qec_last_error());
    }
    ~DecoderCPU() override { qec_decoder_destroy(dec_); }
    DecoderCPU(const DecoderCPU&) = delete;
    DecoderCPU& operator=(const DecoderCPU&) = delete;

    // DecoderCPU::Decode (DecoderCPU.h:317-390)
    ErrorCode Decode(const IntArray1d_h& syndromeX, const IntArray1d_h& syndromeZ, float errorProbability,
                     int maxIterations, IntArray1d_h& outErrorsX, IntArray1d_h& outErrorsZ) override
    {
        std::vector<uint8_t> sx = syndrome_bytes(syndromeX), sz = syndrome_bytes(syndromeZ);
        std::vector<uint8_t> ex(_code.n), ez(_code.n);
        uint8_t flags = 0;
        check(qec_decode_batch(dec_, sx.data(), sz.data(), 1, errorProbability, maxIterations, QEC_STOP_REF, ex.data(),
                               ez.data(), &flags, nullptr, nullptr));
        outErrorsX.assign(ex.begin(), ex.end());
        outErrorsZ.assign(ez.begin(), ez.end());
        return static_cast<ErrorCode>(flags);
    }

    // DecoderCPU::GetStatistics (DecoderCPU.h:392-530): tests (numErrors / nThreads) * nThreads
    // samples, nThreads = the host's hardware threads (the reference's omp_get_max_threads()).
    CodeStatistics GetStatistics(int errorWeight, int numErrors, float errorProbability, int maxIterations,
                                 unsigned int seed) override
    {
        const unsigned hw = std::thread::hardware_concurrency();
        qec_stats s{};
        check(qec_get_statistics(dec_, errorWeight, numErrors, errorProbability, maxIterations, seed, hw ? (int)hw : 1,
                                 &s));
        return CodeStatistics{_code, s.randSeed, s.numErrorsTested, s.numXErrorsTested, s.numZErrorsTested,
                              s.errorWeight, s.corrected, s.syndromeErrorsX, s.syndromeErrorsZ, s.logicalErrors,
                              s.convergenceFailX, s.convergenceFailZ, (long long)s.durationMicroSeconds};
    }
    CodeStatistics GetStatistics(int errorWeight, int numErrors, float errorProbability, int maxIterations) override
    {
        std::random_device rd;
        return GetStatistics(errorWeight, numErrors, errorProbability, maxIterations, rd());
    }

    qec_decoder* handle() { return dec_; }

private:
    qec_decoder* dec_ = nullptr;
    static void check(int rc)
    {
        if (rc != QEC_OK) throw std::string(qec_last_error());
    }
};
