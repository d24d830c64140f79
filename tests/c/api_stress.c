/* Drives most of the C API through many sizes and random operations; built
 * with AddressSanitizer + UndefinedBehaviorSanitizer by `make asan-check`
 * (host build), so leaks, overruns and UB in the front-end, planner, router
 * and host backend show up as failures. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "QuEST.h"
#include "QuEST_debug.h"
#include "quest_amd.h"

static unsigned long long s_rng = 88172645463325252ull;
static unsigned rnd(unsigned n) {
    s_rng ^= s_rng << 13;
    s_rng ^= s_rng >> 7;
    s_rng ^= s_rng << 17;
    return (unsigned)(s_rng % n);
}
static double rndAngle(void) { return (rnd(100000) / 100000.0) * 6.283185307179586; }

static void randomGates(Qureg q, int n, int count) {
    for (int i = 0; i < count; i++) {
        int t = rnd(n), c = rnd(n);
        if (c == t) c = (t + 1) % n;
        switch (rnd(14)) {
            case 0: hadamard(q, t); break;
            case 1: pauliX(q, t); break;
            case 2: pauliY(q, t); break;
            case 3: tGate(q, t); break;
            case 4: rotateX(q, t, rndAngle()); break;
            case 5: rotateZ(q, t, rndAngle()); break;
            case 6: if (n > 1) controlledNot(q, c, t); break;
            case 7: if (n > 1) controlledRotateY(q, c, t, rndAngle()); break;
            case 8: if (n > 1) controlledPhaseFlip(q, c, t); break;
            case 9: {
                Vector v = {0.3, -0.2, 0.9};
                rotateAroundAxis(q, t, rndAngle(), v);
            } break;
            case 10: if (n > 2) {
                int ctrls[2] = {c, (c + 1) % n == t ? (c + 2) % n : (c + 1) % n};
                if (ctrls[1] != t && ctrls[1] != ctrls[0]) {
                    ComplexMatrix2 u = {{0, 1}, {0, 0}, {0, 0}, {0, -1}};
                    multiControlledUnitary(q, ctrls, 2, t, u);
                }
            } break;
            case 11: phaseShift(q, t, rndAngle()); break;
            case 12: if (n > 1) controlledPhaseShift(q, c, t, rndAngle()); break;
            default: sGate(q, t); break;
        }
    }
}

int main(void) {
    QuESTEnv env = createQuESTEnv();
    seedQuEST((unsigned long[]){7, 8, 9}, 3);
    double worst = 0;
    for (int n = 1; n <= 14; n++) {
        Qureg q = createQureg(n, env);
        startRecordingQASM(q);
        initPlusState(q);
        randomGates(q, n, 60 + 10 * n);
        double p = calcTotalProb(q);
        if (fabs(p - 1) > worst) worst = fabs(p - 1);
        for (int t = 0; t < n; t++) (void)calcProbOfOutcome(q, t, rnd(2));
        (void)measure(q, rnd(n));
        Qureg c = createQureg(n, env);
        cloneQureg(c, q);
        (void)calcInnerProduct(c, q);
        (void)getAmp(q, rnd(1u << n));
        destroyQureg(c, env);
        destroyQureg(q, env);
    }
    for (int n = 1; n <= 6; n++) {
        Qureg d = createDensityQureg(n, env);
        Qureg psi = createQureg(n, env);
        initPlusState(psi);
        initPureState(d, psi);
        randomGates(d, n, 40);
        for (int t = 0; t < n; t++) {
            applyOneQubitDephaseError(d, t, 0.1);
            applyOneQubitDepolariseError(d, t, 0.2);
            applyOneQubitDampingError(d, t, 0.3);
            if (n > 1) {
                applyTwoQubitDephaseError(d, t, (t + 1) % n, 0.2);
                applyTwoQubitDepolariseError(d, t, (t + 1) % n, 0.3);
            }
        }
        double tr = calcTotalProb(d);
        if (fabs(tr - 1) > worst) worst = fabs(tr - 1);
        (void)calcPurity(d);
        (void)calcFidelity(d, psi);
        (void)measure(d, rnd(n));
        Qureg d2 = createDensityQureg(n, env);
        initClassicalState(d2, 1);
        addDensityMatrix(d, 0.5, d2);
        destroyQureg(d2, env);
        destroyQureg(psi, env);
        destroyQureg(d, env);
    }
    /* files, checkpoint, fusion off */
    Qureg q = createQureg(5, env);
    initStateDebug(q);
    reportState(q);
    Qureg r = createQureg(5, env);
    char csv[200] = "state_rank_0.csv";  /* the API takes char[200] */
    initStateFromSingleFile(&r, csv, env);
    saveQuregCheckpoint(q, "asan_ckpt");
    loadQuregCheckpoint(r, "asan_ckpt");
    int same = compareStates(q, r, 1e-12);
    setGateFusion(0);
    randomGates(q, 5, 50);
    setGateFusion(1);
    remove("state_rank_0.csv");
    remove("asan_ckpt.0");
    destroyQureg(r, env);
    destroyQureg(q, env);
    destroyQuESTEnv(env);
    printf("api_stress: worst |norm - 1| = %.3g, checkpoint %s\n", worst, same ? "ok" : "MISMATCH");
    return (worst < 1e-10 && same) ? 0 : 1;
}
