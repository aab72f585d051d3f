/*
 * qec_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * Plain-C restatement of the reference's CPU belief-propagation decoder
 * (cantwellc/QEC_LDPC, QEC_LDPC/DecoderCPU.h) and of its Monte-Carlo driver,
 * written from the reference's behaviour, not copied from it.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this file's
 * shared object (oracle/liboracle.so).  The product path (qec_ldpc_amd/,
 * libqecldpc.so) never links or calls it.
 *
 * Parity pin: the reference cannot be built here (it needs cusp/thrust/CUDA
 * headers the image lacks), so this restatement is pinned by the reference's
 * own published artefacts: the seeded CodeStatistics blocks under
 * QEC_LDPC/results/ (all subdirs; extracted to tests/golden/kat.json by
 * tests/golden/make_kat.py).  tests/test_oracle_kat.py reproduces them
 * counter-for-counter.
 *
 * Arithmetic is IEEE binary32 exactly as the reference writes it: build with
 * -O2 -ffp-contract=off and no -ffast-math (x86-64 SSE, FLT_EVAL_METHOD 0).
 * Storage mirrors the reference (dense n x m varNodes / m x n eqNodes and
 * pointer tables) so the timed CPU baseline has the reference's cost shape.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define OC_EXPORT __attribute__((visibility("default")))

/* ErrorCode bits: QEC_LDPC/Decoder.h:14-23 */
enum { OC_SUCCESS = 0, OC_SYN_X = 1, OC_SYN_Z = 2, OC_CONV_X = 4, OC_CONV_Z = 8 };
/* stop rules: 0 = reference (DecoderCPU.h:280-291), 1 = fixed N, 2 = syndrome */
enum { OC_STOP_REF = 0, OC_STOP_FIXED = 1, OC_STOP_SYNDROME = 2 };

typedef struct {
    int J, K, L, P, sigma, tau, n, mX, mZ;
    uint8_t *pcmX; /* mX x n row-major */
    uint8_t *pcmZ; /* mZ x n row-major */
    uint8_t *imp;  /* 2n x 2n row-major (I-P, Quantum_LDPC_Code.h:67-72) */
} oc_code;

/* ------------------------------------------------------------------------- */
/* Code file loader: Quantum_LDPC_Code.h:26-80 (4 lines: J K L P s t / HX / HZ / I-P) */

static const char *next_line(const char *p, const char *end, const char **line_end)
{
    const char *q = p;
    while (q < end && *q != '\n') ++q;
    *line_end = q;
    return q < end ? q + 1 : end;
}

/* stream >> x until failure (Quantum_LDPC_Code.h:28-41); extra values are dropped */
static void parse_ints(const char *p, const char *end, uint8_t *dst, long cap)
{
    long idx = 0;
    while (p < end) {
        while (p < end && (*p == ' ' || *p == '\t' || *p == '\r')) ++p;
        if (p >= end) break;
        int neg = 0;
        if (*p == '-') { neg = 1; ++p; }
        if (p >= end || *p < '0' || *p > '9') break;
        long v = 0;
        while (p < end && *p >= '0' && *p <= '9') v = v * 10 + (*p++ - '0');
        if (idx < cap) dst[idx] = (uint8_t)(neg ? -v : v);
        ++idx;
    }
}

OC_EXPORT void oc_code_free(oc_code *c)
{
    if (!c) return;
    free(c->pcmX); free(c->pcmZ); free(c->imp); free(c);
}

OC_EXPORT oc_code *oc_code_load(const char *path)
{
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;                       /* reference throws (Quantum_LDPC_Code.h:78) */
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    char *buf = (char *)malloc((size_t)sz + 1);
    if (!buf || fread(buf, 1, (size_t)sz, f) != (size_t)sz) { fclose(f); free(buf); return NULL; }
    fclose(f);
    const char *end = buf + sz, *le;
    const char *p = buf;
    oc_code *c = (oc_code *)calloc(1, sizeof(oc_code));
    const char *l1 = p; p = next_line(p, end, &le);
    if (sscanf(l1, "%d %d %d %d %d %d", &c->J, &c->K, &c->L, &c->P, &c->sigma, &c->tau) != 6) {
        free(buf); free(c); return NULL;
    }
    c->n = c->L * c->P; c->mX = c->J * c->P; c->mZ = c->K * c->P;
    c->pcmX = (uint8_t *)calloc((size_t)c->mX * c->n, 1);
    c->pcmZ = (uint8_t *)calloc((size_t)c->mZ * c->n, 1);
    c->imp = (uint8_t *)calloc((size_t)4 * c->n * c->n, 1);
    const char *s;
    s = p; p = next_line(p, end, &le); parse_ints(s, le, c->pcmX, (long)c->mX * c->n);
    s = p; p = next_line(p, end, &le); parse_ints(s, le, c->pcmZ, (long)c->mZ * c->n);
    s = p; p = next_line(p, end, &le); parse_ints(s, le, c->imp, 4L * c->n * c->n);
    free(buf);
    return c;
}

OC_EXPORT void oc_code_info(const oc_code *c, int *out9)
{
    out9[0] = c->J; out9[1] = c->K; out9[2] = c->L; out9[3] = c->P; out9[4] = c->sigma;
    out9[5] = c->tau; out9[6] = c->n; out9[7] = c->mX; out9[8] = c->mZ;
}

/* ------------------------------------------------------------------------- */
/* One sector's BP state: DecoderCPU.h:18-39 (dense arrays + pointer tables). */

typedef struct {
    int n, m, dc, dv;
    const uint8_t *pcm;
    int *eqVar;            /* m*dc  (DecoderCPU.h:41-84, ascending var id)   */
    int *varEq;            /* n*dv  (ascending check id)                      */
    float *eqNodes;        /* m*n,  [eq*n + var]                              */
    float *varNodes;       /* n*m,  [var*m + eq]                              */
    float **eqNodeVarPtrs; /* m*dc -> &varNodes[var*m+eq] (DecoderCPU.h:86-133) */
    float **varNodeEqPtrs; /* n*dv -> &eqNodes[eq*n+var]                      */
} oc_sector;

typedef struct {
    const oc_code *code;
    oc_sector sx, sz;
    int *hd;   /* n scratch */
    int *syn;  /* max(mX,mZ) scratch */
} oc_decoder;

static int sector_init(oc_sector *s, const uint8_t *pcm, int m, int n, int dc, int dv)
{
    s->n = n; s->m = m; s->dc = dc; s->dv = dv; s->pcm = pcm;
    s->eqVar = (int *)malloc(sizeof(int) * (size_t)m * dc);
    s->varEq = (int *)malloc(sizeof(int) * (size_t)n * dv);
    s->eqNodes = (float *)calloc((size_t)m * n, sizeof(float));
    s->varNodes = (float *)calloc((size_t)m * n, sizeof(float));
    s->eqNodeVarPtrs = (float **)malloc(sizeof(float *) * (size_t)m * dc);
    s->varNodeEqPtrs = (float **)malloc(sizeof(float *) * (size_t)n * dv);
    int *vcount = (int *)calloc((size_t)n, sizeof(int));
    /* InitIndexArrays: dense scan, rows in order, columns in order (DecoderCPU.h:51-64) */
    for (int eq = 0; eq < m; ++eq) {
        int k = 0;
        for (int v = 0; v < n; ++v) {
            if (!pcm[(size_t)eq * n + v]) continue;
            if (k >= dc || vcount[v] >= dv) { free(vcount); return -1; } /* irregular code */
            s->eqVar[eq * dc + k++] = v;
            s->varEq[v * dv + vcount[v]++] = eq;
        }
        if (k != dc) { free(vcount); return -1; }
    }
    for (int v = 0; v < n; ++v) if (vcount[v] != dv) { free(vcount); return -1; }
    free(vcount);
    /* InitNodePtrs (DecoderCPU.h:111-132) */
    for (int eq = 0; eq < m; ++eq)
        for (int k = 0; k < dc; ++k)
            s->eqNodeVarPtrs[eq * dc + k] = &s->varNodes[(size_t)s->eqVar[eq * dc + k] * m + eq];
    for (int v = 0; v < n; ++v)
        for (int k = 0; k < dv; ++k)
            s->varNodeEqPtrs[v * dv + k] = &s->eqNodes[(size_t)s->varEq[v * dv + k] * n + v];
    return 0;
}

static void sector_free(oc_sector *s)
{
    free(s->eqVar); free(s->varEq); free(s->eqNodes); free(s->varNodes);
    free(s->eqNodeVarPtrs); free(s->varNodeEqPtrs);
}

OC_EXPORT oc_decoder *oc_decoder_create(const oc_code *c)
{
    oc_decoder *d = (oc_decoder *)calloc(1, sizeof(oc_decoder));
    d->code = c;
    /* DecoderCPU ctor: dc = L, dv = J (X) / K (Z)  (DecoderCPU.h:296-311) */
    if (sector_init(&d->sx, c->pcmX, c->mX, c->n, c->L, c->J) ||
        sector_init(&d->sz, c->pcmZ, c->mZ, c->n, c->L, c->K)) {
        sector_free(&d->sx); sector_free(&d->sz); free(d); return NULL;
    }
    d->hd = (int *)malloc(sizeof(int) * (size_t)c->n);
    d->syn = (int *)malloc(sizeof(int) * (size_t)(c->mX > c->mZ ? c->mX : c->mZ));
    return d;
}

OC_EXPORT void oc_decoder_free(oc_decoder *d)
{
    if (!d) return;
    sector_free(&d->sx); sector_free(&d->sz); free(d->hd); free(d->syn); free(d);
}

/* EqNodeUpdate: DecoderCPU.h:150-186 */
static void eq_node_update(oc_sector *s, const int *syndrome)
{
    const int m = s->m, n = s->n, dc = s->dc;
    for (int eq = 0; eq < m; ++eq) {
        const int first = eq * dc;
        for (int i = 0; i < dc; ++i) {
            const int var = s->eqVar[first + i];
            float product = 1.0f;
            for (int k = 0; k < dc; ++k) {
                if (k == i) continue;
                float value = *s->eqNodeVarPtrs[first + k];
                product *= (1.0f - 2.0f * value);
            }
            const size_t idx = (size_t)eq * n + var;
            if (syndrome[eq])
                s->eqNodes[idx] = (float)(0.5 * (double)(1.0f + product)); /* double in the reference */
            else
                s->eqNodes[idx] = 0.5f * (1.0f - product);
        }
    }
}

/* VarNodeUpdate: DecoderCPU.h:188-229 */
static void var_node_update(oc_sector *s, float errorProbability, int last)
{
    const int m = s->m, n = s->n, dv = s->dv;
    for (int v = 0; v < n; ++v) {
        const size_t firstVarNode = (size_t)v * m;
        const int firstEq = v * dv;
        for (int j = 0; j < dv; ++j) {
            const int eq = s->varEq[firstEq + j];
            float prodP = errorProbability;
            float prodOneMinusP = 1.0f - errorProbability;
            for (int k = 0; k < dv; ++k) {
                if (j == k && !last) continue;
                float p = *s->varNodeEqPtrs[firstEq + k];
                prodOneMinusP *= (1.0f - p);
                prodP *= p;
            }
            s->varNodes[firstVarNode + eq] = prodP / (prodOneMinusP + prodP);
        }
    }
}

/* CheckConvergence: DecoderCPU.h:231-246 (dense scan, zero entries skipped) */
static int check_convergence(const float *est, float high, float low, int n, int m)
{
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < m; ++j) {
            const float e = est[(size_t)i * m + j];
            if (e != 0.0f) {
                if (e > low && e < high) return 0;
            }
        }
    return 1;
}

/* GetSyndromeX/Z: Quantum_LDPC_Code.h:94-124 (dense int MACs, % 2) */
static void dense_syndrome(const uint8_t *pcm, int m, int n, const int *errors, int *syn)
{
    for (int eq = 0; eq < m; ++eq) {
        int x = 0;
        for (int v = 0; v < n; ++v) x += pcm[(size_t)eq * n + v] * errors[v];
        syn[eq] = x % 2;
    }
}

/* hard decision of Decode (DecoderCPU.h:354-373): e[v] = any varNodes[v*m+eq] >= 0.5f */
static void hard_decision(const oc_sector *s, int *e)
{
    for (int v = 0; v < s->n; ++v) {
        e[v] = 0;
        for (int eq = 0; eq < s->m; ++eq)
            if (s->varNodes[(size_t)v * s->m + eq] >= 0.5f) { e[v] = 1; break; }
    }
}

/* BeliefPropogation: DecoderCPU.h:249-292, plus the two extra stop rules.
 * Returns the number of (EqNodeUpdate, VarNodeUpdate) iterations executed. */
static int belief_propagation(oc_decoder *d, oc_sector *s, const int *syndrome, float errorProbability,
                              int maxIterations, int stop)
{
    const float p = 2.0f / 3.0f * errorProbability;  /* DecoderCPU.h:259 */
    const float high = 0.99f, low = 0.01f;
    const size_t numElements = (size_t)s->n * s->m;
    memset(s->varNodes, 0, numElements * sizeof(float));          /* :265 */
    for (int eq = 0; eq < s->m; ++eq)                              /* InitVarNodes :135-148 */
        for (int j = 0; j < s->dc; ++j)
            s->varNodes[(size_t)s->eqVar[eq * s->dc + j] * s->m + eq] = p;
    const int N = maxIterations;
    int converge = 0, iters = 0;
    for (int n = 0; n < N; n++) {
        if (converge) break;                                       /* :282 */
        eq_node_update(s, syndrome);
        var_node_update(s, p, n == N - 1);                         /* prior is p' (:284) */
        ++iters;
        if (stop == OC_STOP_REF) {
            if (n % 10 == 0) converge = check_convergence(s->varNodes, high, low, s->n, s->m);
        } else if (stop == OC_STOP_SYNDROME) {
            hard_decision(s, d->hd);
            dense_syndrome(s->pcm, s->m, s->n, d->hd, d->syn);
            converge = memcmp(d->syn, syndrome, sizeof(int) * (size_t)s->m) == 0;
        }
    }
    return iters;
}

static void q_export(const oc_sector *s, float *q)
{
    for (int eq = 0; eq < s->m; ++eq)
        for (int k = 0; k < s->dc; ++k)
            q[eq * s->dc + k] = s->varNodes[(size_t)s->eqVar[eq * s->dc + k] * s->m + eq];
}

/* Decode: DecoderCPU.h:317-390.  syndromes/outputs are int 0/1 vectors like the reference.
 * iters (optional, 2 ints) receives the iterations executed per sector; qfinal (optional,
 * mX*L + mZ*L floats) the final variable->check messages in [check][slot] order. */
OC_EXPORT int oc_decode(oc_decoder *d, const int *sX, const int *sZ, float errorProbability, int maxIterations,
                        int stop, int *outX, int *outZ, int *iters, float *qfinal)
{
    const oc_code *c = d->code;
    const float high = 0.99f, low = 0.01f;
    int itX = belief_propagation(d, &d->sx, sX, errorProbability, maxIterations, stop);
    int itZ = belief_propagation(d, &d->sz, sZ, errorProbability, maxIterations, stop);
    int code = OC_SUCCESS;
    hard_decision(&d->sx, outX);
    hard_decision(&d->sz, outZ);
    if (!check_convergence(d->sx.varNodes, high, low, c->n, c->mX)) code |= OC_CONV_X;
    if (!check_convergence(d->sz.varNodes, high, low, c->n, c->mZ)) code |= OC_CONV_Z;
    dense_syndrome(c->pcmX, c->mX, c->n, outX, d->syn);
    if (memcmp(d->syn, sX, sizeof(int) * (size_t)c->mX)) code |= OC_SYN_X;
    dense_syndrome(c->pcmZ, c->mZ, c->n, outZ, d->syn);
    if (memcmp(d->syn, sZ, sizeof(int) * (size_t)c->mZ)) code |= OC_SYN_Z;
    if (iters) { iters[0] = itX; iters[1] = itZ; }
    if (qfinal) {
        q_export(&d->sx, qfinal);
        q_export(&d->sz, qfinal + (size_t)c->mX * c->L);
    }
    return code;
}

/* Batch form used by tests and the CPU baseline: one decoder per OpenMP thread,
 * `omp for` over syndromes (the reference's GetStatistics structure, DecoderCPU.h:419-438).
 * u8 in/out, layouts [b][m], [b][n]; iters [b][2]; qfinal [b][mX*L + mZ*L]. */
OC_EXPORT int oc_decode_batch(const oc_code *c, const uint8_t *sX, const uint8_t *sZ, long B,
                              float errorProbability, int maxIterations, int stop,
                              uint8_t *eX, uint8_t *eZ, uint8_t *flags, int32_t *iters, float *qfinal,
                              int nthreads)
{
    const int n = c->n, mX = c->mX, mZ = c->mZ;
    const size_t qper = (size_t)(mX + mZ) * c->L;
    int err = 0;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads)
#endif
    {
        oc_decoder *d = oc_decoder_create(c);
        int *sx = (int *)malloc(sizeof(int) * (size_t)mX), *sz = (int *)malloc(sizeof(int) * (size_t)mZ);
        int *ox = (int *)malloc(sizeof(int) * (size_t)n), *oz = (int *)malloc(sizeof(int) * (size_t)n);
        if (!d) err = 1;
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 8)
#endif
        for (long b = 0; b < B; ++b) {
            if (!d) continue;
            for (int i = 0; i < mX; ++i) sx[i] = sX[b * mX + i];
            for (int i = 0; i < mZ; ++i) sz[i] = sZ[b * mZ + i];
            int it[2];
            int f = oc_decode(d, sx, sz, errorProbability, maxIterations, stop, ox, oz, it,
                              qfinal ? qfinal + b * qper : NULL);
            for (int i = 0; i < n; ++i) { eX[b * n + i] = (uint8_t)ox[i]; eZ[b * n + i] = (uint8_t)oz[i]; }
            if (flags) flags[b] = (uint8_t)f;
            if (iters) { iters[2 * b] = it[0]; iters[2 * b + 1] = it[1]; }
        }
        free(sx); free(sz); free(ox); free(oz);
        oc_decoder_free(d);
    }
    return err ? -1 : 0;
}

/* Dense syndrome of a batch of error vectors (Quantum_LDPC_Code.h:94-124). */
OC_EXPORT void oc_syndrome_batch(const oc_code *c, int sector, const uint8_t *e, long B, uint8_t *s)
{
    const uint8_t *pcm = sector ? c->pcmZ : c->pcmX;
    const int m = sector ? c->mZ : c->mX, n = c->n;
    for (long b = 0; b < B; ++b)
        for (int eq = 0; eq < m; ++eq) {
            int x = 0;
            for (int v = 0; v < n; ++v) x += pcm[(size_t)eq * n + v] * e[b * n + v];
            s[b * m + eq] = (uint8_t)(x % 2);
        }
}

/* CheckLogicalError: Quantum_LDPC_Code.h:126-142 (errors = [x | z], length 2n) */
OC_EXPORT int oc_check_logical(const oc_code *c, const int *errors)
{
    const int N2 = 2 * c->n;
    for (int i = 0; i < N2; ++i) {
        int sum = 0;
        for (int j = 0; j < N2; ++j) sum += c->imp[(size_t)i * N2 + j] * errors[j];
        if (sum % 2 != 0) return 1;
    }
    return 0;
}

/* ------------------------------------------------------------------------- */
/* std::mt19937 (the reference's engine, DecoderCPU.h:394) and the VS2015
 * std::uniform_int_distribution<int>(0, N-1) it was drawn through. */

typedef struct { uint32_t mt[624]; int idx; } oc_mt;

static void mt_seed(oc_mt *g, uint32_t seed)
{
    g->mt[0] = seed;
    for (int i = 1; i < 624; ++i)
        g->mt[i] = 1812433253u * (g->mt[i - 1] ^ (g->mt[i - 1] >> 30)) + (uint32_t)i;
    g->idx = 624;
}

static uint32_t mt_next(oc_mt *g)
{
    if (g->idx >= 624) {
        for (int i = 0; i < 624; ++i) {
            uint32_t y = (g->mt[i] & 0x80000000u) | (g->mt[(i + 1) % 624] & 0x7fffffffu);
            g->mt[i] = g->mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        g->idx = 0;
    }
    uint32_t y = g->mt[g->idx++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

static uint32_t msvc_draw(oc_mt *g, uint32_t N)
{
    for (;;) {
        uint32_t r = mt_next(g);
        if (r / N < 0xFFFFFFFFu / N || 0xFFFFFFFFu % N == N - 1) return r % N;
    }
}

/* The reference's fixed-weight sampler, DecoderCPU.h:449-458: W x (index, type) draws
 * from one shared stream; x=0, y=1, z=2.  Writes COUNT samples [c][n]. */
OC_EXPORT void oc_sample_fixed_weight(uint32_t seed, int W, long count, int n, uint8_t *x, uint8_t *z)
{
    oc_mt g;
    mt_seed(&g, seed);
    memset(x, 0, (size_t)count * n);
    memset(z, 0, (size_t)count * n);
    for (long c = 0; c < count; ++c)
        for (int i = 0; i < W; ++i) {
            int index = (int)msvc_draw(&g, (uint32_t)n);
            int error = (int)msvc_draw(&g, 3u);
            if (error == 0 || error == 1) x[c * n + index] = 1;
            if (error == 2 || error == 1) z[c * n + index] = 1;
        }
}

/* CodeStatistics counters (CodeStatistics.h:5-20), in results-file order. */
typedef struct {
    uint32_t tested, withX, withZ, weight, corrected, synX, synZ, logical, convX, convZ;
} oc_stats;

/* GetStatistics: DecoderCPU.h:392-530.  `tested` samples are drawn (the reference
 * tests (COUNT / nThreads) * nThreads, :426,527).  Counters do not depend on which
 * thread decodes which sample, so the decode is parallel over pre-drawn samples. */
OC_EXPORT int oc_get_statistics(const oc_code *c, int W, long tested, float errorProbability, int maxIterations,
                                uint32_t seed, int nthreads, oc_stats *out)
{
    const int n = c->n, mX = c->mX, mZ = c->mZ;
    const long CHUNK = 8192;
    oc_mt g;
    mt_seed(&g, seed);
    memset(out, 0, sizeof(*out));
    out->weight = (uint32_t)W;
    out->tested = (uint32_t)tested;
    uint8_t *x = (uint8_t *)malloc((size_t)CHUNK * n), *z = (uint8_t *)malloc((size_t)CHUNK * n);
    long withX = 0, withZ = 0, corrected = 0, synX = 0, synZ = 0, logical = 0, convX = 0, convZ = 0;
    for (long base = 0; base < tested; base += CHUNK) {
        long cnt = tested - base < CHUNK ? tested - base : CHUNK;
        memset(x, 0, (size_t)cnt * n);
        memset(z, 0, (size_t)cnt * n);
        for (long s = 0; s < cnt; ++s)
            for (int i = 0; i < W; ++i) {
                int index = (int)msvc_draw(&g, (uint32_t)n);
                int error = (int)msvc_draw(&g, 3u);
                if (error == 0 || error == 1) x[s * n + index] = 1;
                if (error == 2 || error == 1) z[s * n + index] = 1;
            }
#ifdef _OPENMP
        if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads) reduction(+ : withX, withZ, corrected, synX, synZ, logical, convX, convZ)
#endif
        {
            oc_decoder *d = oc_decoder_create(c);
            int *xe = (int *)malloc(sizeof(int) * (size_t)n), *ze = (int *)malloc(sizeof(int) * (size_t)n);
            int *sx = (int *)malloc(sizeof(int) * (size_t)mX), *sz = (int *)malloc(sizeof(int) * (size_t)mZ);
            int *dx = (int *)malloc(sizeof(int) * (size_t)n), *dz = (int *)malloc(sizeof(int) * (size_t)n);
            int *errs = (int *)malloc(sizeof(int) * (size_t)2 * n);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 16)
#endif
            for (long s = 0; s < cnt; ++s) {
                int anyX = 0, anyZ = 0;
                for (int i = 0; i < n; ++i) {
                    xe[i] = x[s * n + i]; ze[i] = z[s * n + i];
                    anyX |= xe[i]; anyZ |= ze[i];
                }
                dense_syndrome(c->pcmX, mX, n, xe, sx);
                dense_syndrome(c->pcmZ, mZ, n, ze, sz);
                withX += anyX; withZ += anyZ;
                int f = oc_decode(d, sx, sz, errorProbability, maxIterations, OC_STOP_REF, dx, dz, NULL, NULL);
                int dEX = (f & OC_SYN_X) != 0, dEZ = (f & OC_SYN_Z) != 0;
                synX += dEX; synZ += dEZ;
                if (!(dEX || dEZ)) {
                    for (int i = 0; i < n; ++i) {
                        errs[i] = (xe[i] + dx[i]) % 2;
                        errs[n + i] = (ze[i] + dz[i]) % 2;
                    }
                    if (oc_check_logical(c, errs)) ++logical; else ++corrected;
                }
                if (f & OC_CONV_X) ++convX;
                if (f & OC_CONV_Z) ++convZ;
            }
            free(xe); free(ze); free(sx); free(sz); free(dx); free(dz); free(errs);
            oc_decoder_free(d);
        }
    }
    free(x); free(z);
    out->withX = (uint32_t)withX; out->withZ = (uint32_t)withZ; out->corrected = (uint32_t)corrected;
    out->synX = (uint32_t)synX; out->synZ = (uint32_t)synZ; out->logical = (uint32_t)logical;
    out->convX = (uint32_t)convX; out->convZ = (uint32_t)convZ;
    return 0;
}
