/* Amplitude damping of one qubit held as a density matrix.
 *
 * Same scenario as the reference's examples/damping_example.c: |+><+| is
 * damped ten times with probability 0.1 and the state is printed after
 * every step.  Expected: rho_11 = 0.5 * 0.9^k, coherences 0.5 * 0.9^(k/2).
 */
#include <stdio.h>

#include "QuEST.h"

int main(void) {
    QuESTEnv env = createQuESTEnv();
    printf("-------------------------------------------------------\n");
    printf("QuEST (MI355X build) damping example: one qubit, ten damping steps of p = 0.1\n");
    printf("-------------------------------------------------------\n");

    Qureg rho = createDensityQureg(1, env);
    initPlusState(rho);
    printf("\ninitial state:\n");
    reportStateToScreen(rho, env, 0);

    for (int step = 1; step <= 10; step++) {
        applyOneQubitDampingError(rho, 0, 0.1);
        printf("\nafter %d damping step%s:\n", step, step > 1 ? "s" : "");
        reportStateToScreen(rho, env, 0);
    }
    printf("\nP(|1>) = %.10f (expected %.10f)\n", calcProbOfOutcome(rho, 0, 1), 0.5 * 0.3486784401);

    destroyQureg(rho, env);
    destroyQuESTEnv(env);
    return 0;
}
