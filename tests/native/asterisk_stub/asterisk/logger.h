/* TEST STUB: ast_log to stderr. */
#ifndef TFP_TEST_AST_LOGGER_H
#define TFP_TEST_AST_LOGGER_H
#define LOG_ERROR 4, __FILE__, __LINE__, __func__
#define LOG_WARNING 3, __FILE__, __LINE__, __func__
#define LOG_NOTICE 2, __FILE__, __LINE__, __func__
#define LOG_VERBOSE 1, __FILE__, __LINE__, __func__
void ast_log(int level, const char* file, int line, const char* function, const char* fmt, ...)
    __attribute__((format(printf, 5, 6)));
#endif
