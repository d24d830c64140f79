/* The fork's 30-qubit benchmark program (zhaozzz-160/QuEST
 * tutorial_example.c): apply the 490-gate random circuit, then write
 * P(q_i = 1) for every qubit and the first 10 amplitudes, and report the wall
 * time of the whole run (the fork quotes an *estimated* 3783.93 s for it).
 *
 * The circuit is read from a text file (one API call per line,
 * examples/data/fork_circuit_30q.txt) rather than compiled in.
 *
 *   random_circuit_benchmark [circuit.txt] [numQubits] [probs.dat] [amps.dat]
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>

#include "QuEST.h"

static double wallTime(void) {
    struct timeval t;
    gettimeofday(&t, NULL);
    return (double)t.tv_sec + 1e-6 * (double)t.tv_usec;
}

static int applyLine(Qureg q, char* line) {
    char name[64];
    int a = 0, b = 0;
    double x = 0;
    if (line[0] == '#' || line[0] == '\n' || line[0] == 0) return 0;
    if (sscanf(line, "%63s", name) != 1) return 0;
    const char* rest = line + strlen(name);
    if (!strcmp(name, "hadamard") && sscanf(rest, "%d", &a) == 1) hadamard(q, a);
    else if (!strcmp(name, "pauliX") && sscanf(rest, "%d", &a) == 1) pauliX(q, a);
    else if (!strcmp(name, "pauliY") && sscanf(rest, "%d", &a) == 1) pauliY(q, a);
    else if (!strcmp(name, "pauliZ") && sscanf(rest, "%d", &a) == 1) pauliZ(q, a);
    else if (!strcmp(name, "sGate") && sscanf(rest, "%d", &a) == 1) sGate(q, a);
    else if (!strcmp(name, "tGate") && sscanf(rest, "%d", &a) == 1) tGate(q, a);
    else if (!strcmp(name, "rotateX") && sscanf(rest, "%d %lf", &a, &x) == 2) rotateX(q, a, x);
    else if (!strcmp(name, "rotateY") && sscanf(rest, "%d %lf", &a, &x) == 2) rotateY(q, a, x);
    else if (!strcmp(name, "rotateZ") && sscanf(rest, "%d %lf", &a, &x) == 2) rotateZ(q, a, x);
    else if (!strcmp(name, "controlledNot") && sscanf(rest, "%d %d", &a, &b) == 2) controlledNot(q, a, b);
    else if (!strcmp(name, "controlledPauliY") && sscanf(rest, "%d %d", &a, &b) == 2) controlledPauliY(q, a, b);
    else if (!strcmp(name, "controlledRotateX") && sscanf(rest, "%d %d %lf", &a, &b, &x) == 3)
        controlledRotateX(q, a, b, x);
    else if (!strcmp(name, "controlledRotateY") && sscanf(rest, "%d %d %lf", &a, &b, &x) == 3)
        controlledRotateY(q, a, b, x);
    else if (!strcmp(name, "controlledRotateZ") && sscanf(rest, "%d %d %lf", &a, &b, &x) == 3)
        controlledRotateZ(q, a, b, x);
    else {
        fprintf(stderr, "unrecognised circuit line: %s", line);
        exit(1);
    }
    return 1;
}

int main(int argc, char** argv) {
    const char* circuit = argc > 1 ? argv[1] : "examples/data/fork_circuit_30q.txt";
    const int numQubits = argc > 2 ? atoi(argv[2]) : 30;
    const char* probsPath = argc > 3 ? argv[3] : "probs.dat";
    const char* ampsPath = argc > 4 ? argv[4] : "stateVector.dat";

    FILE* fc = fopen(circuit, "r");
    if (!fc) {
        fprintf(stderr, "cannot open %s\n", circuit);
        return 1;
    }
    QuESTEnv env = createQuESTEnv();
    const double t0 = wallTime();
    Qureg q = createQureg(numQubits, env);

    char line[512];
    int gates = 0;
    while (fgets(line, sizeof line, fc)) gates += applyLine(q, line);
    fclose(fc);

    FILE* fp = env.rank == 0 ? fopen(probsPath, "w") : NULL;
    FILE* fv = env.rank == 0 ? fopen(ampsPath, "w") : NULL;
    for (int i = 0; i < numQubits; i++) {
        qreal p = calcProbOfOutcome(q, i, 1);
        if (fp) fprintf(fp, "Probability for q[%2d]==1 : %lf    \n", i, (double)p);
    }
    for (int i = 0; i < 10; i++) {
        Complex amp = getAmp(q, i);
        if (fv) fprintf(fv, "Amplitude of %dth state vector: %12.6f,%12.6f\n", i, (double)amp.real, (double)amp.imag);
    }
    const double t1 = wallTime();
    if (fp) fclose(fp);
    if (fv) fclose(fv);
    if (env.rank == 0) {
        printf("%d qubits, %d gates, %d probabilities, 10 amplitudes\n", numQubits, gates, numQubits);
        printf("Complete the simulation takes time %12.6f seconds.\n", t1 - t0);
    }
    destroyQureg(q, env);
    destroyQuESTEnv(env);
    return 0;
}
