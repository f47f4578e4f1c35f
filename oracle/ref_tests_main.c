/*
 * ref_tests_main.c -- own driver for the reference's FEC known-answer tests
 * (sim_test/fec_test/test_func.c:8-334).  The reference main.c
 * (sim_test/fec_test/main.c:4-13) enables only test_flex_receiver(80, 4);
 * this driver runs all of them.  Linked two ways by oracle/Makefile:
 *   _ref/ref_fec_test        with the reference flex_fec_xor.c   (the oracle)
 *   _ref/fec_test_on_razor   with librazor_fec.so instead        (drop-in proof)
 * Both must print identical output (tests/test_dropin.py).
 */
#include <stdint.h>
#include <stdio.h>

#include "test_func.h"

int main(int argc, const char* argv[])
{
    (void)argc;
    (void)argv;
    setvbuf(stdout, NULL, _IONBF, 0);
    test_fec_xor();
    test_num_fec();
    test_flex_sender(20);
    test_flex_sender(80);
    test_flex_receiver(20, 2);
    test_flex_receiver(80, 4);
    return 0;
}
