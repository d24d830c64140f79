/* Bernstein-Vazirani style oracle check on 9 qubits (qubit 0 = ancilla),
 * the scenario of the reference's examples/bernstein_vazirani_circuit.c:
 * the secret s = 0b10001 is written onto qubits 1..8 by CNOTs from the
 * flipped ancilla, and the probability of reading s back is printed
 * (expected 1.000000).
 */
#include <stdio.h>

#include "QuEST.h"

int main(void) {
    const int numQubits = 9;
    const int secret = (1 << 4) + 1;

    QuESTEnv env = createQuESTEnv();
    Qureg q = createQureg(numQubits, env);
    initZeroState(q);

    pauliX(q, 0);
    for (int qb = 1; qb < numQubits; qb++)
        if ((secret >> (qb - 1)) & 1) controlledNot(q, 0, qb);

    double success = 1.0;
    for (int qb = 1; qb < numQubits; qb++) success *= calcProbOfOutcome(q, qb, (secret >> (qb - 1)) & 1);
    printf("solution reached with probability %f\n", success);

    destroyQureg(q, env);
    destroyQuESTEnv(env);
    return success > 1 - 1e-9 ? 0 : 1;
}
