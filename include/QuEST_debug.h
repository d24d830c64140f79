/* Debug / test-only API (reference: QuEST/src/QuEST_debug.h:23-53,
 * definitions QuEST.c:699-726).  Exported so that test harnesses can build
 * fixtures that bypass the physical-state checks of the public API. */
#ifndef QUEST_DEBUG_H
#define QUEST_DEBUG_H

#include "QuEST.h"

#ifdef __cplusplus
extern "C" {
#endif

/* qubit `qubitId` fixed to `outcome`, all other qubits uniform. */
void initStateOfSingleQubit(Qureg* qureg, int qubitId, int outcome);
/* amp[i] = (2i/10) + i (2i+1)/10 with i the global index (non-physical). */
void initStateDebug(Qureg qureg);
/* Read "re, im" lines (lines starting with '#' skipped). */
void initStateFromSingleFile(Qureg* qureg, char filename[200], QuESTEnv env);
/* 1 iff every real and imaginary part differs by at most precision. */
int compareStates(Qureg qureg1, Qureg qureg2, qreal precision);
/* Overwrite every element of a density matrix (flat column-major order). */
void setDensityAmps(Qureg qureg, qreal* reals, qreal* imags);
/* QuEST_PREC the library was built with. */
int getQuEST_PREC(void);

#ifdef __cplusplus
}
#endif

#endif /* QUEST_DEBUG_H */
