/*
 * qec_ldpc.h -- C ABI of libqecldpc.so, the MI355X (gfx950) belief-propagation
 * decoder for quasi-cyclic CSS quantum LDPC codes.
 *
 * Plain C: opaque handles, plain pointers and sizes, int status codes
 * (0 = ok, < 0 = error, text in qec_last_error()).  No HIP or torch types
 * appear in any signature; streams are passed as `void*` (a hipStream_t or NULL).
 *
 * Each entry point names the reference interface it replaces
 * (cantwellc/QEC_LDPC, paths relative to the repository root).
 *
 * Threading: a qec_code is immutable after creation and may be shared.  Calls on
 * one qec_decoder are serialised by the caller (like one DecoderCPU per OpenMP
 * thread, QEC_LDPC/DecoderCPU.h:431); distinct decoders may be driven from
 * distinct host threads.
 *
 * Streams: the device-pointer (_dev) entry points enqueue on the caller's stream and
 * return without synchronising.  A decoder's workspace (dispatch order, flag-merge
 * words) is reused by every launch; a launch on a stream other than the previous
 * launch's first waits for that launch (an event), so calls on one decoder from
 * several streams are ordered, not concurrent.  For concurrency use one decoder per
 * stream.  Every entry point restores the caller's current HIP device.
 */
#ifndef QEC_LDPC_H
#define QEC_LDPC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QEC_LDPC_ABI_VERSION 4

/* status codes */
enum {
    QEC_OK = 0,
    QEC_ERR_ARG = -1,          /* bad argument (null pointer, out-of-range size) */
    QEC_ERR_IO = -2,           /* file missing/unreadable ("Unable to find code file", Quantum_LDPC_Code.h:78) */
    QEC_ERR_FORMAT = -3,       /* malformed code file */
    QEC_ERR_UNSUPPORTED = -4,  /* code shape the GPU engine does not handle */
    QEC_ERR_HIP = -5,          /* HIP runtime error / no GPU */
    QEC_ERR_NOMEM = -6
};

/* ErrorCode bit flags, identical to Decoder::ErrorCode (QEC_LDPC/Decoder.h:14-23) */
enum {
    QEC_SUCCESS = 0,
    QEC_SYNDROME_FAIL_X = 1 << 0,
    QEC_SYNDROME_FAIL_Z = 1 << 1,
    QEC_SYNDROME_FAIL_XZ = QEC_SYNDROME_FAIL_X | QEC_SYNDROME_FAIL_Z,
    QEC_CONVERGENCE_FAIL_X = 1 << 2,
    QEC_CONVERGENCE_FAIL_Z = 1 << 3,
    QEC_CONVERGENCE_FAIL_XZ = QEC_CONVERGENCE_FAIL_X | QEC_CONVERGENCE_FAIL_Z
};

/* BP stop rules */
enum {
    QEC_STOP_REF = 0,      /* DecoderCPU::BeliefPropogation (DecoderCPU.h:280-291): convergence test at n % 10 == 0 */
    QEC_STOP_FIXED = 1,    /* exactly maxIterations iterations (the headline "fixed BP iters") */
    QEC_STOP_SYNDROME = 2  /* stop once the hard decision satisfies the syndrome (per sector) */
};

enum { QEC_SECTOR_X = 0, QEC_SECTOR_Z = 1 };

/* GPU engines behind one decoder handle */
enum {
    QEC_ENGINE_AUTO = 0,       /* wave-circulant if the code has an instantiated kernel, else sparse-graph */
    QEC_ENGINE_CIRCULANT = 1,  /* wave-circulant: circulant-permutation QC codes, P <= 64 (bp_decode.hip) */
    QEC_ENGINE_SPARSE = 2,     /* sparse-graph: any code DecoderCPU accepts (regular, dc = L, dv = J / K) */
    QEC_ENGINE_CPU = 3         /* host threads, device -1 (DecoderCPU's drop-in; cpu_engine.cpp) */
};

typedef struct qec_code qec_code;
typedef struct qec_decoder qec_decoder;

/* CodeStatistics (QEC_LDPC/CodeStatistics.h:5-20) counters */
typedef struct {
    uint32_t randSeed;
    uint32_t numErrorsTested;
    uint32_t numXErrorsTested;
    uint32_t numZErrorsTested;
    uint32_t errorWeight;
    uint32_t corrected;
    uint32_t syndromeErrorsX;
    uint32_t syndromeErrorsZ;
    uint32_t logicalErrors;
    uint32_t convergenceFailX;
    uint32_t convergenceFailZ;
    int64_t durationMicroSeconds;
} qec_stats;

/* ---- diagnostics ---------------------------------------------------------- */
const char* qec_last_error(void);  /* message of the last failing call on this thread */
int qec_abi_version(void);         /* QEC_LDPC_ABI_VERSION */
/* Build id of this library: a hash of the sources and flags it was compiled from (the same for every
 * rebuild of the same tree); rocprofv3 profiles are stamped with it (tools/gpu/pmc_summary.py). */
const char* qec_build_id(void);

/* ---- code model ----------------------------------------------------------- */
/* Replaces Quantum_LDPC_Code::createFromFile (QEC_LDPC/Quantum_LDPC_Code.h:26-80):
 * 4-line text file "J K L P sigma tau" / HX / HZ / I-P.  NULL on error. */
qec_code* qec_code_load(const char* path);
/* Replaces the QC_LDPC_CSS(J,K,L,P,sigma,tau) generator (QEC_LDPC/QEC_LDPC_CSS.cu:5-131).
 * Generated codes carry no I-P matrix (the reference never generates one). */
qec_code* qec_code_generate(int J, int K, int L, int P, int sigma, int tau);
int qec_code_free(qec_code* code);
/* J K L P sigma tau n numEqsX numEqsZ (Quantum_LDPC_Code.h:10-20) into out[9] */
int qec_code_params(const qec_code* code, int* out9);
/* circulant shift of every P x P block, J x L (X) or K x L (Z), row-major;
 * returns QEC_ERR_UNSUPPORTED if the code is not a circulant-permutation QC code */
int qec_code_exponents(const qec_code* code, int sector, int* out);
/* dense parity-check matrix pcmX / pcmZ (m x n, 0/1) */
int qec_code_pcm(const qec_code* code, int sector, uint8_t* out);
/* "[J=..,K=..,L=..,P=..,s=..,t=..][[n=..,k=..]]" (Quantum_LDPC_Code.h:145-150) */
int qec_code_describe(const qec_code* code, char* buf, size_t len);
/* Quantum_LDPC_Code::GetSyndromeX/Z (Quantum_LDPC_Code.h:94-124) for B error vectors,
 * e: B x n (0/1) -> s: B x m (host memory) */
int qec_code_syndrome(const qec_code* code, int sector, const uint8_t* e, size_t B, uint8_t* s);
/* Quantum_LDPC_Code::CheckLogicalError (Quantum_LDPC_Code.h:126-142) on the
 * residual [ex | ez] of B samples; out[b] = 1 if logical error */
int qec_code_check_logical(const qec_code* code, const uint8_t* ex, const uint8_t* ez, size_t B, uint8_t* out);

/* ---- decoder (DecoderGPU, QEC_LDPC/DecoderGPU.h:11-281) ------------------- */
/* Replaces DecoderGPU(Quantum_LDPC_Code) (DecoderGPU.h:117-130) and, with device = -1,
 * DecoderCPU(Quantum_LDPC_Code) (DecoderCPU.h:16-39): the CPU engine, host threads over
 * edge-major tables, bit-identical decisions; it serves the host-buffer entry points and
 * qec_get_statistics (the _dev entry points and qec_monte_carlo need a GPU and fail with
 * QEC_ERR_UNSUPPORTED).  device >= 0 = HIP device ordinal.  max_batch sizes the
 * device-pointer workspace up front: the _dev decode entry points then allocate nothing
 * for B <= max_batch and may be captured into a graph.  Larger batches grow it on
 * demand (an error while the stream is being captured). */
qec_decoder* qec_decoder_create(const qec_code* code, int device, size_t max_batch);
/* Same with an explicit engine (QEC_ENGINE_*).  QEC_ENGINE_CIRCULANT fails with
 * QEC_ERR_UNSUPPORTED when the code has no wave-circulant kernel; QEC_ENGINE_SPARSE fails
 * for an irregular code (DecoderCPU's index tables assume row weight L and column weight
 * J / K, DecoderCPU.h:41-84). */
qec_decoder* qec_decoder_create_engine(const qec_code* code, int device, size_t max_batch, int engine);
int qec_decoder_destroy(qec_decoder* dec);
/* A decoder over several devices (the reference's sample-parallel loop, DecoderCPU.h:419-438,
 * spread over GPUs; main.cu:79,101 unchanged): one single-device part per entry of devices[]
 * (a device may appear more than once: two parts then share it).  The host-pointer entry
 * points (qec_decode_batch, qec_decode_batch_packed) split the batch into contiguous shards,
 * one per part, decoded concurrently; qec_get_statistics and qec_monte_carlo shard their
 * samples the same way and sum the parts' counters (bit-identical to one device: the counters
 * do not depend on sample order).  Options apply to every part.  The _dev entry points need
 * a single-device handle: call them on qec_decoder_part(dec, k).  Every ordinal must be >= 0
 * (QEC_ERR_ARG otherwise: a group is GPU-only). */
qec_decoder* qec_decoder_create_multi(const qec_code* code, const int* devices, int ndevices, size_t max_batch);
int qec_decoder_num_parts(const qec_decoder* dec);      /* 1 for a single-device decoder */
qec_decoder* qec_decoder_part(qec_decoder* dec, int k); /* part k (the handle itself for k = 0 of a single one) */
int qec_decoder_device(const qec_decoder* dec);         /* HIP device ordinal (of part 0 for a group) */
/* Decoder options (no reference analogue: DecoderCPU has none).
 *   QEC_OPT_HARD_PATHS (default 1): once every message of a sector is exactly +0 or 1.0 the
 *     wave-circulant kernels switch to the exact hard-message forms of the check and variable
 *     updates (bp_decode.hip, check_pass_hard / var_pass).  Outputs are bit-identical either
 *     way; 0 forces the full arithmetic every iteration (for measurement).
 *   QEC_OPT_CYCLE_JUMP (default 1; needs QEC_OPT_HARD_PATHS): once a hard sector whose
 *     variables all carry equal messages takes an iteration that leaves every variable's inputs
 *     unchanged, the remaining iterations provably alternate between the two states just seen
 *     (bp_decode.hip, cycle_end), so the kernel jumps to the sector's last iteration.
 *     Bit-identical either way; 0 runs the remaining hard iterations one by one (for
 *     measurement).
 *   QEC_OPT_SCHEDULE (default 1): dispatch order of the wave-circulant launch.  Two small
 *     kernels (a counting sort) order the batch by syndrome weight and the decode waves take syndromes heaviest
 *     first, so the rare syndromes that run every iteration in full arithmetic start early
 *     instead of extending the launch (schedule.hip); a sector-split launch orders each sector's
 *     waves by that sector's weight.  Outputs are written at each syndrome's
 *     own index and are bit-identical either way.  0 = batch order, 1 = sorted when
 *     4096 <= B <= 2^22 (codes with one syndrome per wave, P > 32: 4096 <= B <= 2^19, above which
 *     the pass costs more than it saves), 2 = sorted when B <= 2^22, 3 = as 2 but with the one-launch
 *     local order for B <= 2^18 short-row codes (each chunk sorted in LDS, chunks interleaved by rank;
 *     measured slower than the global sort at P7 65 536, kept for experiments), 4 = as 2 but the
 *     global sort in one launch with a software grid barrier for up to 128 chunks (measured slower).
 *     The workspace (10 B per syndrome + 1 MiB) is allocated
 *     by qec_decoder_create for max_batch and grown on demand by larger calls.
 *   QEC_OPT_SECTOR_SPLIT (default 1): the X and Z sectors of a syndrome are decoded by two
 *     waves instead of one after the other (halves the longest wave).  The launch then zeroes
 *     flags[] first and each sector ORs in its bits.  Bit-identical either way.  0 = off,
 *     1 = the kernel variant's measured choice (P7: split waves up to 2^20 syndromes, above 2^19 only
 *     with the per-sector dispatch order; P61: sector launches from 2^18 on under the fixed stop, at 2^20
 *     under the reference stop, at 2^20 and p >= 0.03 under the syndrome stop), 2 = on where the variant
 *     has split kernels (the two shipped codes),
 *     3 = sector launches: two launches on the caller's stream, sector X then
 *     sector Z, each kernel compiled (and its registers allocated) for its own sector only; the Z
 *     launch ORs its flags into the byte the X launch stored (shipped codes; elsewhere as 0).
 *   QEC_OPT_PHASE_STATS (default 0; measurement only, shipped codes): launches an instrumented
 *     copy of the kernel whose iters[] output packs, per sector, the iterations executed in each
 *     phase instead of their count: soft | hard << 8 | agreed << 16 | jumped << 24 (soft: full
 *     arithmetic; hard: hard-message forms; agreed: the agreement path; jumped: skipped by the
 *     cycle jump; each field mod 256).  Decisions and flags are unchanged.
 *   QEC_OPT_TRIAGE (default 1; shipped codes, syndrome stop with N >= 2 on the Monte-Carlo
 *     pipeline's bit-row syndromes, i.e. qec_monte_carlo): a triage kernel decides iteration 0 of
 *     64 syndromes per wave from the syndrome patterns (triage.hip); the sectors it does not stop
 *     are compacted into lists the decode kernel then decodes (list mode).  Bit-identical either
 *     way.  0 = off (every sector in the decode kernel), 1 = when p <= 0.01 (above it most
 *     sectors go on and the ordered decode of the whole batch is faster), 2 = always, 3 = as 1
 *     without the fused form.  Fused form (1, 2; depolarising qec_monte_carlo runs): sampler,
 *     syndromes, triage and the finished samples' statistics in one kernel, so only the samples
 *     with a sector that goes on reach HBM (list-mode decode, then their statistics).
 *   QEC_OPT_LAST_PATH (read only; qec_decoder_set_option refuses it): the launch sequence the
 *     handle's last decode call enqueued, as QEC_PATH_* bits (0 before the first decode), so a test
 *     can assert which kernels its comparison went through.
 *   QEC_OPT_MC_DECODE_TIME (default 1): qec_monte_carlo times its decode kernels with an event pair
 *     per batch (qec_mc_result.decodeSeconds).  0: no events between its launches (each costs the
 *     GPU a few microseconds, ~5 % of a 2^20-sample batch at p = 0.001) and decodeSeconds = 0;
 *     counters unchanged. */
enum { QEC_OPT_HARD_PATHS = 1, QEC_OPT_CYCLE_JUMP = 2, QEC_OPT_SCHEDULE = 3, QEC_OPT_SECTOR_SPLIT = 4,
       QEC_OPT_PHASE_STATS = 5, QEC_OPT_TRIAGE = 6, QEC_OPT_LAST_PATH = 7, QEC_OPT_MC_DECODE_TIME = 8 };
enum {
    QEC_PATH_ORDERED = 1,          /* dispatch order pass (schedule.hip) */
    QEC_PATH_SECTOR_ORDER = 2,     /* ... in the per-sector form (each sector's waves by its own weight) */
    QEC_PATH_SPLIT_WAVES = 4,      /* X and Z sectors in separate waves of one launch */
    QEC_PATH_SECTOR_LAUNCHES = 8,  /* an X launch, then a Z launch */
    QEC_PATH_TRIAGE = 16,          /* iteration-0 triage + list-mode decode */
    QEC_PATH_BIT_ROWS = 32,        /* bit-row syndromes in */
    QEC_PATH_SPARSE = 64,          /* sparse-graph engine */
    QEC_PATH_RECORDS = 128         /* packed decision records out */
};
int qec_decoder_set_option(qec_decoder* dec, int option, int value);
int qec_decoder_get_option(const qec_decoder* dec, int option, int* value);
/* which kernel variant serves this code: writes a short name (e.g. "wave-circulant P=61 G=1") */
int qec_decoder_describe(const qec_decoder* dec, char* buf, size_t len);

/* Batched Decoder::Decode (QEC_LDPC/Decoder.h:40-41, semantics of
 * DecoderCPU::Decode, DecoderCPU.h:317-390) on HOST buffers; synchronous.
 *   sX: B x numEqsX, sZ: B x numEqsZ   syndromes (0/1 bytes)
 *   eX, eZ: B x n                      decoded error estimates (0/1 bytes)
 *   flags: B                           ErrorCode bits per syndrome pair
 *   iters: B x 2 (optional)            BP iterations executed (X, Z)
 *   q_final: B x (numEqsX+numEqsZ) x L (optional) final variable->check messages,
 *            [check][slot] with slots in ascending variable order (X block first)
 * errorProbability / maxIterations as in Decode; stop = QEC_STOP_*. */
int qec_decode_batch(qec_decoder* dec, const uint8_t* sX, const uint8_t* sZ, size_t B,
                     float errorProbability, int maxIterations, int stop,
                     uint8_t* eX, uint8_t* eZ, uint8_t* flags, int32_t* iters, float* q_final);
/* Same on DEVICE buffers (same layouts), enqueued on `stream` (hipStream_t or NULL),
 * asynchronous: no host synchronisation, no allocation (graph-capturable). */
int qec_decode_batch_dev(qec_decoder* dec, const uint8_t* sX, const uint8_t* sZ, size_t B,
                         float errorProbability, int maxIterations, int stop,
                         uint8_t* eX, uint8_t* eZ, uint8_t* flags, int32_t* iters, float* q_final,
                         void* stream);
/* Bit-packed output (SURVEY.md 8(d)'s I/O model): the decode kernel writes one decision record
 * per syndrome instead of eX / eZ / flags: records is B x QEC_RECORD_BYTES(n) bytes, per syndrome
 * eX packed (ceil(n/8) bytes, bit j of byte k = qubit 8k + j, padding bits 0), then eZ packed,
 * then the ErrorCode flags byte.  Same decisions bit for bit as the byte form. */
#define QEC_RECORD_BYTES(n) (2 * (((n) + 7) / 8) + 1)
int qec_decode_batch_packed_dev(qec_decoder* dec, const uint8_t* sX, const uint8_t* sZ, size_t B,
                                float errorProbability, int maxIterations, int stop,
                                uint8_t* records, int32_t* iters, float* q_final, void* stream);
/* The same with bit-row syndromes (the Monte-Carlo pipeline's layout, 72 instead of 549 bytes per
 * P61 syndrome): sXbits [B][ceil(numEqsX / 32)] and sZbits [B][ceil(numEqsZ / 32)] 32-bit words,
 * bit c of a row = check c (bit c % 32 of word c / 32).  Wave-circulant engine only
 * (QEC_ERR_UNSUPPORTED otherwise).  Under the syndrome stop this is the entry point that takes
 * the triage (QEC_OPT_TRIAGE) when no final messages are requested. */
int qec_decode_bits_packed_dev(qec_decoder* dec, const uint32_t* sXbits, const uint32_t* sZbits, size_t B,
                               float errorProbability, int maxIterations, int stop,
                               uint8_t* records, int32_t* iters, float* q_final, void* stream);
/* Host-buffer form of the packed decode (synchronous). */
int qec_decode_batch_packed(qec_decoder* dec, const uint8_t* sX, const uint8_t* sZ, size_t B,
                            float errorProbability, int maxIterations, int stop,
                            uint8_t* records, int32_t* iters);

/* ---- Monte-Carlo caller side (DecoderCPU::GetStatistics, DecoderCPU.h:392-530) */
/* The reference's fixed-weight sampler (DecoderCPU.h:448-459, RandomErrorGenerator.h:31-44):
 * one mt19937(seed) stream, VS2015 uniform_int_distribution, W x (index, type) draws per
 * sample.  x, z: count x n (0/1). */
int qec_sample_fixed_weight(uint32_t seed, int W, size_t count, int n, uint8_t* x, uint8_t* z);
/* Decoder::GetStatistics(errorWeight, numErrors, errorProbability, maxIterations, seed)
 * (Decoder.h:44-47): samples numErrors errors exactly as the reference does, decodes them on
 * the GPU (reference stop rule) and fills the CodeStatistics counters.  The reference tests
 * (numErrors / nThreads) * nThreads samples; pass nThreads = 1 to test all numErrors. */
int qec_get_statistics(qec_decoder* dec, int errorWeight, int numErrors, float errorProbability,
                       int maxIterations, uint32_t seed, int nThreads, qec_stats* out);

/* ---- Monte-Carlo on the device (the GetStatistics loop, batched) ---- */
/* counters in device order for qec_statistics_dev */
enum { QEC_MC_WITHX, QEC_MC_WITHZ, QEC_MC_SYNX, QEC_MC_SYNZ, QEC_MC_LOGICAL, QEC_MC_CORRECTED, QEC_MC_CONVX,
       QEC_MC_CONVZ, QEC_MC_NCOUNTERS,
       /* qec_statistics_packed_dev with iters: BP iterations executed, summed per sector */
       QEC_MC_ITERX = QEC_MC_NCOUNTERS, QEC_MC_ITERZ, QEC_MC_NCOUNTERS_ALL };

typedef struct {
    uint64_t tested, withX, withZ, synX, synZ, logical, corrected, convX, convZ;
    uint64_t iterationsX, iterationsZ; /* BP iterations executed, summed over samples */
    double decodeSeconds;             /* decode-kernel time (HIP events), summed over batches */
    double totalSeconds;              /* wall time of the call */
} qec_mc_result;

/* i.i.d. depolarising errors for samples [start, start+B) of stream `seed` (device buffers
 * x, z: B x n).  Each qubit is hit with probability thr / 2^32, thr = floor(p 2^32) (saturated),
 * independently, drawn as a walk over the gaps between hits: sample b reads 32-bit words from
 * Philox4x32-10 calls k = 0, 1, ... (counter (b lo, b hi, k, 0x6A9C0DE5), key (seed lo, seed hi),
 * word 4k + j = output word j of call k); u = next word skips G = #{g in 1..n : u < T[g]} qubits,
 * T[g] = floor(q^g 2^32), q = 1 - thr / 2^32 (q^g by right-to-left binary exponentiation in IEEE
 * double); a qubit still inside the sample is then hit, of type floor(3 w / 2^32) of the next word
 * w: 0 = X, 1 = Y, 2 = Z (Y sets both bits).  Any shard of the index space can be drawn alone. */
int qec_sample_depolarizing_dev(qec_decoder* dec, uint64_t seed, uint64_t start, size_t B, float p, uint8_t* x,
                                uint8_t* z, void* stream);
/* Fused front end: the depolarising errors of qec_sample_depolarizing_dev (same stream, same
 * bits) go straight to their syndromes (GetSyndromeX/Z, Quantum_LDPC_Code.h:94-124) without
 * leaving the chip: sX B x numEqsX, sZ B x numEqsZ, and optionally errp B x 2 ceil(n/8), the
 * errors bit-packed in the decision-record layout (x bits then z bits) for
 * qec_statistics_packed_dev.  One wave per sample. */
int qec_sample_syndrome_dev(qec_decoder* dec, uint64_t seed, uint64_t start, size_t B, float p, uint8_t* sX,
                            uint8_t* sZ, uint8_t* errp, void* stream);
/* GetSyndromeX/Z (Quantum_LDPC_Code.h:94-124) of device error vectors: x, z B x n -> sX B x numEqsX, sZ B x numEqsZ */
int qec_syndrome_dev(qec_decoder* dec, const uint8_t* x, const uint8_t* z, size_t B, uint8_t* sX, uint8_t* sZ,
                     void* stream);
/* The CodeStatistics counters of a decoded device batch (DecoderCPU.h:464-521: errors present,
 * syndrome fails, I-P logical check when neither syndrome failed, convergence fails), ADDED to
 * the device array counters[QEC_MC_NCOUNTERS] (uint64). */
int qec_statistics_dev(qec_decoder* dec, const uint8_t* x, const uint8_t* z, const uint8_t* eX, const uint8_t* eZ,
                       const uint8_t* flags, size_t B, uint64_t* counters, void* stream);
/* The same counters from packed errors (qec_sample_syndrome_dev's errp) and packed decision
 * records (qec_decode_batch_packed_dev), ADDED to counters[QEC_MC_NCOUNTERS], or, with iters
 * (B x 2, nullable) given, to counters[QEC_MC_NCOUNTERS_ALL] including the iteration sums. */
int qec_statistics_packed_dev(qec_decoder* dec, const uint8_t* errp, const uint8_t* records, const int32_t* iters,
                              size_t B, uint64_t* counters, void* stream);
/* Decision records for gathering a sharded batch to one rank (the decoded
 * vectors travel bit-packed): out is B x (2 ceil(n/8) + 1) bytes, per syndrome eX packed
 * (bit j of byte k = qubit 8k + j), then eZ packed, then the ErrorCode flags byte.  Device
 * buffers, enqueued on `stream`. */
int qec_pack_decisions_dev(qec_decoder* dec, const uint8_t* eX, const uint8_t* eZ, const uint8_t* flags, size_t B,
                           uint8_t* out, void* stream);
/* A whole Monte-Carlo run on the device: `count` depolarising samples from `start` of stream
 * `seed`, in batches of `batch`: fused sample + syndrome -> packed decode (stop rule `stop`) ->
 * statistics with iteration sums, all on the device with no per-batch host synchronisation.
 * A multi-device decoder shards [start, start + count) contiguously over its parts.
 * Synchronous; fills *out (decodeSeconds: decode-kernel time, the largest over parts). */
int qec_monte_carlo(qec_decoder* dec, uint64_t seed, uint64_t start, uint64_t count, float errorProbability,
                    int maxIterations, int stop, size_t batch, qec_mc_result* out);

#ifdef __cplusplus
}
#endif
#endif /* QEC_LDPC_H */
