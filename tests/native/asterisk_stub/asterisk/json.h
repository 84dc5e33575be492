/* TEST STUB: a minimal ast_json (objects, arrays, integers, reals, strings, null), the subset of
 * Asterisk's json.h API the shim and catalog call. */
#ifndef TFP_TEST_AST_JSON_H
#define TFP_TEST_AST_JSON_H
#include <stddef.h>
#include <stdint.h>
struct ast_json;
struct ast_json* ast_json_object_create(void);
struct ast_json* ast_json_array_create(void);
struct ast_json* ast_json_null(void);
struct ast_json* ast_json_integer_create(intmax_t v);
struct ast_json* ast_json_real_create(double v);
struct ast_json* ast_json_string_create(const char* s);
int ast_json_object_set(struct ast_json* obj, const char* key, struct ast_json* value); /* steals value */
struct ast_json* ast_json_object_get(struct ast_json* obj, const char* key);
int ast_json_array_append(struct ast_json* array, struct ast_json* value);              /* steals value */
size_t ast_json_array_size(const struct ast_json* array);
struct ast_json* ast_json_array_get(const struct ast_json* array, size_t index);
intmax_t ast_json_integer_get(const struct ast_json* v);
double ast_json_real_get(const struct ast_json* v);
const char* ast_json_string_get(const struct ast_json* v);
void ast_json_unref(struct ast_json* v);
#endif
