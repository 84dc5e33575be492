/* fp_catalog.h — what shim/fp_handler_tfp.c needs from the Asterisk side's catalog.
 *
 * In the module these are the reference's own functions over its SQLite DB (db_ctx_handler.c),
 * exported from fp_handler.c instead of being static there:
 *   fpc_db_init / fpc_db_term           fp_handler.c:68-108 (init_database + load / backup)
 *   fpc_create_audio_list_info          fp_handler.c:479-530 (MD5 dedup + INSERT audio_list)
 *   fpc_get_audio_list_info             fp_handler.c:832-855
 *   fpc_delete_audio_list_info          fp_handler.c:115-159 (both DELETEs)
 *   fpc_store_fingerprints              fp_handler.c:538-575 (the audio_fingerprint rows, now
 *                                       written in one transaction: they back up the GPU index)
 *   fpc_for_each_fingerprint_clip       the restored audio_fingerprint table, one clip at a time
 *                                       (tiresias_amd/dbio.py's query), for the GPU index
 *   fp_generate_uuid                    fp_handler.c:1097-1109
 */
#ifndef FP_CATALOG_H
#define FP_CATALOG_H

#include <stdbool.h>
#include <stdint.h>

struct ast_json;

bool fpc_db_init(void);
bool fpc_db_term(void);
/* 1 created, 0 already enrolled (same context and file hash), < 0 error */
int fpc_create_audio_list_info(const char* context, const char* filename, const char* uuid);
struct ast_json* fpc_get_audio_list_info(const char* uuid); /* {uuid, name, context, hash} or NULL */
bool fpc_delete_audio_list_info(const char* uuid);
/* m1/m2: "%f" micro-units, INT32_MIN for NULL (TFP_NULL_MICRO) */
bool fpc_store_fingerprints(const char* context, const char* uuid, const int32_t* m1, const int32_t* m2,
                            int64_t n);
typedef bool (*fpc_clip_rows_cb)(void* arg, const char* uuid, const int32_t* m1, const int32_t* m2, int64_t n);
bool fpc_for_each_fingerprint_clip(fpc_clip_rows_cb cb, void* arg);
char* fp_generate_uuid(void);

#endif
