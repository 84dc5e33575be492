/* TEST STUB: Asterisk's allocation wrappers. */
#ifndef TFP_TEST_AST_UTILS_H
#define TFP_TEST_AST_UTILS_H
#include <stdlib.h>
#include <string.h>
#define ast_malloc(n) malloc(n)
#define ast_calloc(n, m) calloc((n), (m))
#define ast_free(p) free(p)
#define ast_realloc(p, n) realloc((p), (n))
#define ast_strdup(s) strdup(s)
#endif
