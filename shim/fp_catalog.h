/* fp_catalog.h — the catalog half of the module's engine facade (src/fp_handler.h:13-38), over
 * SQLite, implemented in shim/fp_catalog.c. shim/fp_handler_tfp.c holds the hot half (enrolment
 * and search on the GPU); together they replace the reference's fp_handler.c and db_ctx_handler.c.
 *
 * The state is the reference's: one in-memory SQLite DB (fp_handler.c:30, :680) with the tables of
 * init_database (:673-756), filled at fp_init from the backup file by ATTACH + "insert into main.T
 * select * from backup.T" (db_ctx_load_db_data, db_ctx_handler.c:750-772, :827-841) and copied back
 * to it page by page at fp_term (db_ctx_backup, db_ctx_handler.c:673-717). The audio_fingerprint
 * rows are still written, one per frame with the "%f" text of each value (db_ctx_insert_basic,
 * db_ctx_handler.c:413-556, reals :479-481; an absent key -> NULL), so the backup file is the one the
 * reference module reads and writes; the GPU index is loaded from it at fp_init.
 *
 *   fpc_db_init / fpc_db_term        fp_handler.c:68-108 (init_database + load / backup)
 *   fpc_create_audio_list_info       fp_handler.c:479-530 (MD5 dedup per context + INSERT audio_list)
 *   fpc_get_audio_list_info          fp_handler.c:832-855
 *   fpc_delete_audio_list_info       fp_handler.c:115-159 (both DELETEs)
 *   fpc_store_fingerprints           fp_handler.c:538-575 (the audio_fingerprint INSERTs, one
 *                                    transaction per clip)
 *   fpc_load_fingerprints            the restored audio_fingerprint table grouped by clip, for one
 *                                    tfp_index_add_batch
 * and the reference's control-plane entry points themselves (fp_handler.h:16-23, :37-38):
 *   fp_create_context_list_info, fp_delete_context_list_info, fp_get_context_lists_all,
 *   fp_get_context_list_info, fp_get_audio_lists_all, fp_get_audio_lists_by_contextname,
 *   fp_generate_uuid, fp_create_hash.
 * Thread-safe: one lock around every catalog operation. */
#ifndef FP_CATALOG_H
#define FP_CATALOG_H

#include <stdbool.h>
#include <stdint.h>

struct ast_json;

#define FPC_DEF_BACKUP_DATABASE "/var/lib/asterisk/third-party/tiresias/audio_recongition.db" /* fp_handler.c:31 */

/* The backup file (default FPC_DEF_BACKUP_DATABASE); before fpc_db_init. */
void fpc_set_backup_path(const char* path);
bool fpc_db_init(void);
/* Backup to the file, then close. False when the backup could not be written (closed anyway). */
bool fpc_db_term(void);
/* Close without writing the backup (a failed fp_init). */
void fpc_db_close(void);

/* 1 created, 0 already enrolled (same context and file hash), < 0 error */
int fpc_create_audio_list_info(const char* context, const char* filename, const char* uuid);
/* The same; when the file is already enrolled (0), existing[len] receives that row's uuid. */
int fpc_create_audio_list_info_ex(const char* context, const char* filename, const char* uuid, char* existing,
		size_t len);
struct ast_json* fpc_get_audio_list_info(const char* uuid); /* {uuid, name, context, hash} or NULL */
bool fpc_delete_audio_list_info(const char* uuid);
/* m1/m2: "%f" micro-units, INT32_MIN for NULL (TFP_NULL_MICRO) */
bool fpc_store_fingerprints(const char* context, const char* uuid, const int32_t* m1, const int32_t* m2,
                            int64_t n);

/* The audio_fingerprint table by clip (uuid order, frame rows in insertion order): clip c's rows are
 * [frame_offsets[c], frame_offsets[c + 1]) of m1 / m2. Release with fpc_rows_free. */
typedef struct fpc_rows {
	int32_t nclips;
	char** uuids;
	int64_t* frame_offsets;
	int32_t* m1;
	int32_t* m2;
} fpc_rows;
bool fpc_load_fingerprints(fpc_rows* out);
void fpc_rows_free(fpc_rows* rows);

/* fp_handler.h:16-23, :37-38 */
bool fp_create_context_list_info(const char* name, const char* directory, bool replace);
bool fp_delete_context_list_info(const char* name);
struct ast_json* fp_get_context_lists_all(void);
struct ast_json* fp_get_context_list_info(const char* name);
struct ast_json* fp_get_audio_lists_all(void);
struct ast_json* fp_get_audio_lists_by_contextname(const char* name);
char* fp_generate_uuid(void);
char* fp_create_hash(const char* filename);

/* implemented by the hot half (shim/fp_handler_tfp.c): fp_delete_context_list_info removes each of
 * the context's audio files through it, as the reference does (fp_handler.c:1066-1084) */
bool fp_delete_audio_list_info(const char* uuid);

#endif
