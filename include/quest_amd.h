/* MI355X-native extensions to the QuEST API.
 *
 * Everything in QuEST.h behaves as in the reference.  These functions expose
 * what the MI355X design adds: deferred, fused gate execution; explicit
 * flush/sync; runtime statistics; host mirrors and zero-copy device access
 * for interop (e.g. with PyTorch); and error handling without exit().
 */
#ifndef QUEST_AMD_H
#define QUEST_AMD_H

#include "QuEST.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Called instead of exit() on invalid input; the API call then returns
 * without modifying any state.  Pass NULL to restore print-and-exit. */
typedef void (*QuESTErrorHandler)(int errorCode, const char* message, const char* function);
void setQuESTErrorHandler(QuESTErrorHandler handler);

/* Gate fusion: unitaries are queued per register and applied in as few
 * passes over the state as possible (LDS-tiled passes on the GPU).  Any
 * operation that reads the state flushes the queue first, so results are
 * identical with fusion on or off.  Default: on (env QUEST_FUSION=0: off). */
void setGateFusion(int enabled);
int getGateFusion(void);
/* Maximum number of qubits spanned by one fused pass (0 = default). */
void setFusionMaxQubits(int numQubits);

/* Tuning knobs.  Any build: "fuse_blocks" (compose gate pairs into 4x4
 * blocks before scheduling), "verify" (debug: re-run every fused flush op by
 * op on a shadow copy of the state and exit with a report if the results
 * differ; env QUEST_VERIFY=1, tolerance QUEST_VERIFY_TOL), "plan_max_ops"
 * (most ops one fused pass takes, 0 = no limit; env QUEST_PLAN_MAX_OPS),
 * "wave_relabel", "wave_lane_order" (0 need order, 1 lanes by position, 2
 * wave bits latest-needed), "wave_shadow" (debug: check every wave pass
 * against the host emulation; env QUEST_WAVE_SHADOW=1).  HIP build: "direct_kernels" (LDS-free kernel for a pass
 * holding one gate), "tile_mode" (0 op by op, 1 register phases, 2 dense
 * blocks, 3 wave tiles), "tile_qubits", "tile_wg_per_cu", "wave_wg_per_cu",
 * "wave_tile_map" (XCD-aware tile order of the wave kernel),
 * "direct_layout" (0 grid-stride, 1 looping runs, 2 one run per workgroup),
 * "direct_low_to_tile" (1: gates on bits inside a 128-byte line go to the tile
 * pass).  Returns 1 if the key is known.  Also settable at start via
 * QUEST_DIRECT_KERNELS / QUEST_TILE_MODE / QUEST_TILE_QUBITS /
 * QUEST_TILE_WG_PER_CU / ...
 *
 * Start-up only (HIP build): QUEST_IM_GAP (bytes between a register's re and
 * im arrays when they are 1 GiB or larger, default 8 GiB, taken only when a
 * tenth of the device stays free), QUEST_ALLOC_MODE (0 two allocations, 1
 * joint with QUEST_IM_OFFSET, 2 physically contiguous, 3 mapped address range
 * with QUEST_IM_DIST; experiments), QUEST_CACHED_STATE_MB (states up to this
 * size, default 128 MiB, use plain instead of non-temporal accesses in the
 * unfused kernels), QUEST_SYNC_SPIN=1 (spinning host waits), and for several
 * ranks QUEST_COMM (rccl default, ipc / socket for ranks sharing one GPU) and
 * QUEST_RCCL_SHARED_GPU=1 (RCCL itself with several ranks on one GPU: a host
 * id per rank, RCCL's network transport).  Any build: QUEST_DEPHASE_DIAG=0
 * keeps dephasing channels in channel form instead of diagonal ops;
 * QUEST_FRONT_FLUSH (queued ops at which the first wave pass is planned and
 * launched while the program keeps issuing gates, default 512, 0 = off);
 * QUEST_DIAG_PHASES (lone diagonal gates as phase ops: 0 never, 1 always,
 * 2 default: queues of at most 4 ops per qubit); QUEST_WAVE_CMIN_SEARCH=1
 * (per window, 6 or 7 always-resident low positions by trial plans). */
int setQuESTTuning(const char* key, int value);
/* Current value of a tuning knob (into *value); returns 1 if the key is known. */
int getQuESTTuning(const char* key, int* value);

/* Submit every queued operation of the register to the device (async). */
void flushQureg(Qureg qureg);
/* flushQureg + wait for the device. */
void syncQureg(Qureg qureg);

/* Host mirror (Qureg.stateVec), allocated only when QUEST_HOST_MIRROR=1 at
 * createQureg time on the HIP build. */
void copyStateToGPU(Qureg qureg);
void copyStateFromGPU(Qureg qureg);

/* Copy this rank's chunk to / from caller-owned buffers that live where the
 * state lives (device memory on the HIP build).  Register must be in the
 * canonical qubit layout (it is made canonical first). */
void copyChunkToBuffers(Qureg qureg, qreal* re, qreal* im);
void copyChunkFromBuffers(Qureg qureg, const qreal* re, const qreal* im);

/* Collective read of the amplitudes [startInd, startInd + numAmps) of a
 * state-vector (or of the flattened density matrix) into host arrays on
 * every rank; the counterpart of setAmps. */
void getAmps(Qureg qureg, long long int startInd, qreal* reals, qreal* imags, long long int numAmps);

/* Binary checkpoint: every rank streams its (canonical) chunk to
 * "<path>.<rank>" behind a 64-byte header.  Collective; returns 1 on success
 * everywhere.  A checkpoint written by R ranks restores on any number of ranks
 * (same qubits, register type and precision, else E_CHECKPOINT_MISMATCH). */
int saveQuregCheckpoint(Qureg qureg, const char* path);
int loadQuregCheckpoint(Qureg qureg, const char* path);

/* Per-rank device memory a register of numQubitsInStateVec qubits needs on
 * numRanks ranks (0: the current number), in bytes: out = {state (re + im of the
 * chunk), exchange slice buffers of distributed swaps, scratch, total}.
 * createQureg / createDensityQureg check the total against the free device
 * memory (E_OUT_OF_MEMORY with this breakdown); QUEST_DEVICE_MEM_MB overrides
 * the free amount. */
void getQuregMemoryPlan(int numQubitsInStateVec, int numRanks, long long out[4]);

/* Diagnostic: drive the device transport's code paths (HIP build: RCCL with a
 * one-rank communicator -- pipelined exchange on the communication stream,
 * scalar allreduce / broadcast, allgather, async-error polling) and check the
 * data.  Single-process jobs only.  Returns 1 if everything matched; a
 * description goes to report. */
int runCommSelfTest(char* report, int reportLen);

/* Diagnostic: the per-rank footprint of a numQubitsInStateVec-qubit register
 * on numRanks ranks, shown on THIS single-process job's device next to what it
 * already holds (e.g. a register of the per-rank size): the exchange buffers of
 * the plan's largest all-to-all swap are allocated, a one-rank transport
 * communicator is brought up and the pipelined exchange runs through them.
 * Returns 1 if the data matched and the buffers are the plan's; the report
 * gives the plan and the free device memory before / with the buffers / with
 * the communicator up. */
int runFootprintCheck(int numQubitsInStateVec, int numRanks, char* report, int reportLen);

/* Restore the canonical qubit layout after distributed qubit remapping. */
void canonicaliseQureg(Qureg qureg);
/* physical bit position of each logical qubit of the state-vector */
void getQubitLayout(Qureg qureg, int* physicalOfLogical);

typedef struct QuESTStats {
    long long opsQueued;      /* elementary ops accepted by the backend */
    long long passes;         /* passes over the state (kernel launches of gate kernels) */
    long long fusedOps;       /* ops applied inside multi-op passes */
    long long swaps;          /* global<->local qubit swaps (distributed) */
    long long bytesExchanged; /* bytes sent to other ranks */
    long long reductions;     /* reduction kernels */
    long long verifiedFlushes; /* flushes checked op by op (QUEST_VERIFY=1 / tuning "verify") */
    long long wavePasses;     /* passes run by the register-resident wave-tile engine */
    long long waveOps;        /* ops of those passes, including transpositions */
    long long waveTransposes; /* cross-lane transpositions among them */
    long long relabels;       /* X/Y-like gates on rank qubits applied by relabelling chunks (no data moved) */
    long long globalDiags;    /* diagonal one-qubit gates on rank qubits applied as per-rank scalings */
    long long flushes;        /* backend queue flushes (each planned into fused passes) */
    long long marginalPasses; /* one-pass computations of every qubit's marginal (calcProbOfOutcome cache) */
    long long waveShadowChecks;     /* wave passes compared with the host emulation (tuning "wave_shadow") */
    long long waveShadowMismatches; /* ... that differed from it */
    long long permutedOps;    /* inner products / addDensityMatrix of registers in different qubit layouts,
                                 computed by the permuted kernels without a relayout */
    long long relayouts;      /* canonicalisations that moved data (getAmps, file IO, ... after relabelling) */
    long long restoreRounds;  /* concurrent rounds of whole-chunk exchanges restoring the chunk placement */
    long long swapMicros;     /* device time of the qubit swaps (HIP: events on the compute stream; reading waits for them) */
    long long overlappedSwaps;  /* swaps run on a stream of their own, next to gate passes (QUEST_SWAP_OVERLAP) */
    long long overlappedPasses; /* passes started on the part of the chunk a swap in flight leaves in place */
    long long layoutAligns;   /* swaps / chunk restores before which this rank moved its local qubits to rank 0's positions */
    long long placementProbes; /* re / im placements measured by the allocation probe (HIP; 1 when a remembered one was taken) */
} QuESTStats;
void getQuESTStats(QuESTStats* stats);
void resetQuESTStats(void);

/* Name of the compiled backend: "HIP" (gfx950) or "CPU". */
const char* getQuESTBackend(void);
/* The inter-rank transport in use (RCCL / socket / single process). */
const char* getQuESTTransport(void);

/* Seed array used by seedQuESTDefault on this rank (after broadcast). */
void getQuESTSeeds(unsigned long* seeds, int* numSeeds);

#ifdef __cplusplus
}
#endif

#endif /* QUEST_AMD_H */
