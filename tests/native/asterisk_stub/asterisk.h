/* TEST STUB (tests/native/asterisk_stub): the few Asterisk declarations shim/fp_handler_tfp.c
 * uses, so the shim compiles and runs outside Asterisk in tests/test_shim.py. Not product code. */
#ifndef TFP_TEST_ASTERISK_H
#define TFP_TEST_ASTERISK_H
#include <stdbool.h>
#include <stddef.h>
#endif
