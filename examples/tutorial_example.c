/* 3-qubit walkthrough of the QuEST API (same circuit as the reference's
 * examples/tutorial_example.c:4-91, whose documented output is
 * P(|111>) = 0.498751 and P(q2 = 1) = 0.749178, examples/README.md:146-156).
 * Build:  make examples  (CPU)   or   make build/examples/tutorial_example_hip */
#include <stdio.h>

#include "QuEST.h"

int main(void) {
    QuESTEnv env = createQuESTEnv();

    printf("-------------------------------------------------------\n");
    printf("QuEST-for-MI355X tutorial: a 3-qubit circuit\n");
    printf("-------------------------------------------------------\n");

    Qureg qubits = createQureg(3, env);
    initZeroState(qubits);

    printf("\nThis is our environment:\n");
    reportQuregParams(qubits);
    reportQuESTEnv(env);

    hadamard(qubits, 0);
    controlledNot(qubits, 0, 1);
    rotateY(qubits, 2, .1);

    int all3[3] = {0, 1, 2};
    multiControlledPhaseFlip(qubits, all3, 3);

    ComplexMatrix2 u;
    u.r0c0 = (Complex){.real = .5, .imag = .5};
    u.r0c1 = (Complex){.real = .5, .imag = -.5};
    u.r1c0 = (Complex){.real = .5, .imag = -.5};
    u.r1c1 = (Complex){.real = .5, .imag = .5};
    unitary(qubits, 0, u);

    Complex a = {.real = .5, .imag = .5};
    Complex b = {.real = .5, .imag = -.5};
    compactUnitary(qubits, 1, a, b);

    Vector v = {.x = 1, .y = 0, .z = 0};
    rotateAroundAxis(qubits, 2, 3.14 / 2, v);

    controlledCompactUnitary(qubits, 0, 1, a, b);

    int first2[2] = {0, 1};
    multiControlledUnitary(qubits, first2, 2, 2, u);

    printf("\nCircuit output:\n");
    qreal prob = getProbAmp(qubits, 7);
    printf("Probability amplitude of |111>: %f\n", prob);

    prob = calcProbOfOutcome(qubits, 2, 1);
    printf("Probability of qubit 2 being in state 1: %f\n", prob);

    int outcome = measure(qubits, 0);
    printf("Qubit 0 was measured in state %d\n", outcome);

    outcome = measureWithStats(qubits, 2, &prob);
    printf("Qubit 2 collapsed to %d with probability %f\n", outcome, prob);

    destroyQureg(qubits, env);
    destroyQuESTEnv(env);
    return 0;
}
