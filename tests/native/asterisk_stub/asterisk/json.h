/* TEST STUB: a minimal ast_json (objects, arrays, integers, reals, strings, null), the subset of
 * Asterisk's json.h API the shim and catalog call. */
#ifndef TFP_TEST_AST_JSON_H
#define TFP_TEST_AST_JSON_H
#include <stddef.h>
#include <stdint.h>
struct ast_json;
enum ast_json_type { AST_JSON_OBJECT, AST_JSON_ARRAY, AST_JSON_STRING, AST_JSON_INTEGER, AST_JSON_REAL, AST_JSON_TRUE,
                     AST_JSON_FALSE, AST_JSON_NULL };
struct ast_json_error;
/* jansson's json_loads(input, 0, ...) as Asterisk calls it: an array or object at the top, else NULL */
struct ast_json* ast_json_load_string(const char* input, struct ast_json_error* error);
enum ast_json_type ast_json_typeof(const struct ast_json* value);
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
