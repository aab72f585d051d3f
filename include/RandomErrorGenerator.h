// RandomErrorGenerator.h -- the reference's fixed-weight X/Y/Z sampler
// (QEC_LDPC/RandomErrorGenerator.h:5-45, inlined at QEC_LDPC/DecoderCPU.h:448-459).
// The draws go through VS2015's uniform_int_distribution algorithm (the one the
// published seeds were produced with), not the host library's,
// so a seed reproduces the reference's error sequence on any compiler.
// Fix vs reference: `seed` is the seed the engine was actually seeded with (the
// reference reported mt19937::default_seed while seeding from random_device).
#pragma once
#include <cstdint>
#include <random>
#include <vector>

class RandomErrorGenerator {
public:
    unsigned int seed;

    explicit RandomErrorGenerator(int numVars) : RandomErrorGenerator(numVars, std::random_device{}()) {}
    RandomErrorGenerator(int numVars, unsigned int s) : seed(s), numVars_(numVars), engine_(s) {}

    // W draws of (index, type); type x=0, y=1, z=2 (RandomErrorGenerator.h:31-44)
    void GenerateError(std::vector<int>& xErrors, std::vector<int>& zErrors, int errorWeight)
    {
        for (int i = 0; i < errorWeight; ++i) {
            const uint32_t index = draw((uint32_t)numVars_);
            const uint32_t error = draw(3u);
            if (error == 0 || error == 1) xErrors[index] = 1;
            if (error == 2 || error == 1) zErrors[index] = 1;
        }
    }

private:
    int numVars_;
    std::mt19937 engine_;

    uint32_t draw(uint32_t N)  // uniform_int_distribution<int>(0, N-1), VS2015 rejection rule
    {
        for (;;) {
            const uint32_t r = (uint32_t)engine_();
            if (r / N < 0xFFFFFFFFu / N || 0xFFFFFFFFu % N == N - 1) return r % N;
        }
    }
};
