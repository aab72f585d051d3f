// DecoderGPU.h -- the reference's named GPU slot (QEC_LDPC/DecoderGPU.h:11-281),
// now backed by the MI355X engine in libqecldpc.so.  Same class name, same
// constructor and method signatures, so QEC_LDPC/main.cu's loop switches engines by
// replacing `DecoderCPU decoder(code);` with `DecoderGPU decoder(code);`.
//
// Added: DecodeBatch / DecodeBatchPacked (the batched boundary the GPU engine is built for), and
// a multi-device constructor: DecoderGPU(code, {0, 1, ..., 7}) spreads GetStatistics' samples
// (and batched decodes) over the listed GPUs with counters identical to one device
// (qec_decoder_create_multi).  Decode() keeps the reference's one-syndrome-pair semantics (a
// batch of one: one launch, copies and a synchronisation per call -- loop DecodeBatch instead).
#pragma once
#include <cstdint>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "Decoder.h"

class DecoderGPU : public Decoder {
public:
    // DecoderGPU.h:117; device = HIP ordinal
    explicit DecoderGPU(Quantum_LDPC_Code code, int device = 0) : Decoder(code)
    {
        dec_ = qec_decoder_create(_code.handle(), device, 0);
        if (!dec_) throw std::string(qec_last_error());
    }
    // several GPUs of this node (a device may repeat); every call shards its samples over them
    DecoderGPU(Quantum_LDPC_Code code, const std::vector<int>& devices) : Decoder(code)
    {
        dec_ = qec_decoder_create_multi(_code.handle(), devices.data(), (int)devices.size(), 0);
        if (!dec_) throw std::string(qec_last_error());
    }
    ~DecoderGPU() override { qec_decoder_destroy(dec_); }
    DecoderGPU(const DecoderGPU&) = delete;
    DecoderGPU& operator=(const DecoderGPU&) = delete;

    // Decoder::Decode (Decoder.h:40-41) with DecoderCPU::Decode semantics (DecoderCPU.h:317-390)
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

    // B syndrome pairs at once: sX [B*numEqsX], sZ [B*numEqsZ] -> eX, eZ [B*n], flags [B]
    void DecodeBatch(const std::vector<uint8_t>& sX, const std::vector<uint8_t>& sZ, size_t B, float errorProbability,
                     int maxIterations, int stopRule, std::vector<uint8_t>& eX, std::vector<uint8_t>& eZ,
                     std::vector<uint8_t>& flags)
    {
        eX.resize(B * _code.n);
        eZ.resize(B * _code.n);
        flags.resize(B);
        check(qec_decode_batch(dec_, sX.data(), sZ.data(), B, errorProbability, maxIterations, stopRule, eX.data(),
                               eZ.data(), flags.data(), nullptr, nullptr));
    }

    // B syndrome pairs -> packed decision records [B * QEC_RECORD_BYTES(n)] (eX bits, eZ bits, flags)
    void DecodeBatchPacked(const std::vector<uint8_t>& sX, const std::vector<uint8_t>& sZ, size_t B,
                           float errorProbability, int maxIterations, int stopRule, std::vector<uint8_t>& records)
    {
        records.resize(B * QEC_RECORD_BYTES(_code.n));
        check(qec_decode_batch_packed(dec_, sX.data(), sZ.data(), B, errorProbability, maxIterations, stopRule,
                                      records.data(), nullptr));
    }

    // DecoderGPU::GetStats (DecoderGPU.h:193-228): statistics over pre-generated flat
    // COUNT x n error arrays (the reference's stub decoded nothing; this one decodes).
    CodeStatistics GetStats(int errorWeight, int numErrors, float errorProbability, int maxIterations, int seed,
                            std::vector<int>& xErrors, std::vector<int>& zErrors)
    {
        const int n = _code.n;
        const size_t B = (size_t)numErrors;
        std::vector<uint8_t> x(B * n), z(B * n), sx(B * _code.numEqsX), sz(B * _code.numEqsZ);
        for (size_t k = 0; k < B * n; ++k) { x[k] = (uint8_t)(xErrors[k] & 1); z[k] = (uint8_t)(zErrors[k] & 1); }
        check(qec_code_syndrome(_code.handle(), 0, x.data(), B, sx.data()));
        check(qec_code_syndrome(_code.handle(), 1, z.data(), B, sz.data()));
        std::vector<uint8_t> ex, ez, fl;
        DecodeBatch(sx, sz, B, errorProbability, maxIterations, QEC_STOP_REF, ex, ez, fl);
        std::vector<uint8_t> rx(n), rz(n);
        CodeStatistics st{_code, (unsigned)seed, (unsigned)numErrors, 0, 0, (unsigned)errorWeight, 0, 0, 0, 0, 0, 0, 0};
        for (size_t b = 0; b < B; ++b) {
            bool ax = false, az = false;
            for (int v = 0; v < n; ++v) { ax |= x[b * n + v] != 0; az |= z[b * n + v] != 0; }
            st.numXErrorsTested += ax;
            st.numZErrorsTested += az;
            const bool dEX = fl[b] & SYNDROME_FAIL_X, dEZ = fl[b] & SYNDROME_FAIL_Z;
            st.syndromeErrorsX += dEX;
            st.syndromeErrorsZ += dEZ;
            if (!(dEX || dEZ)) {
                for (int v = 0; v < n; ++v) {
                    rx[v] = (x[b * n + v] + ex[b * n + v]) % 2;
                    rz[v] = (z[b * n + v] + ez[b * n + v]) % 2;
                }
                uint8_t le = 0;
                check(qec_code_check_logical(_code.handle(), rx.data(), rz.data(), 1, &le));
                if (le) ++st.logicalErrors; else ++st.corrected;
            }
            st.convergenceFailX += (fl[b] & CONVERGENCE_FAIL_X) != 0;
            st.convergenceFailZ += (fl[b] & CONVERGENCE_FAIL_Z) != 0;
        }
        return st;
    }

    // Decoder::GetStatistics (DecoderCPU.h:392-530 semantics; errors drawn from the same
    // mt19937(seed) stream as the reference, decoded in GPU batches)
    CodeStatistics GetStatistics(int errorWeight, int numErrors, float errorProbability, int maxIterations,
                                 unsigned int seed) override
    {
        qec_stats s{};
        check(qec_get_statistics(dec_, errorWeight, numErrors, errorProbability, maxIterations, seed, 1, &s));
        return CodeStatistics{_code, s.randSeed, s.numErrorsTested, s.numXErrorsTested, s.numZErrorsTested,
                              s.errorWeight, s.corrected, s.syndromeErrorsX, s.syndromeErrorsZ, s.logicalErrors,
                              s.convergenceFailX, s.convergenceFailZ, (long long)s.durationMicroSeconds};
    }
    CodeStatistics GetStatistics(int errorWeight, int numErrors, float errorProbability, int maxIterations) override
    {
        std::random_device rd;
        return GetStatistics(errorWeight, numErrors, errorProbability, maxIterations, rd());
    }

    std::string Describe() const
    {
        char buf[256];
        qec_decoder_describe(dec_, buf, sizeof buf);
        return buf;
    }
    qec_decoder* handle() { return dec_; }

private:
    qec_decoder* dec_ = nullptr;
    static void check(int rc)
    {
        if (rc != QEC_OK) throw std::string(qec_last_error());
    }
};
