/* TEST STUB: a minimal ast_json (object of integer / string members). */
#ifndef TFP_TEST_AST_JSON_H
#define TFP_TEST_AST_JSON_H
#include <stdint.h>
struct ast_json;
struct ast_json* ast_json_object_create(void);
struct ast_json* ast_json_integer_create(intmax_t v);
struct ast_json* ast_json_string_create(const char* s);
int ast_json_object_set(struct ast_json* obj, const char* key, struct ast_json* value); /* steals value */
struct ast_json* ast_json_object_get(struct ast_json* obj, const char* key);
intmax_t ast_json_integer_get(const struct ast_json* v);
const char* ast_json_string_get(const struct ast_json* v);
void ast_json_unref(struct ast_json* v);
#endif
