/* fp_catalog.c — the catalog half of the engine facade over SQLite (shim/fp_catalog.h).
 *
 * Same tables, SQL effects and return conventions as the reference's fp_handler.c /
 * db_ctx_handler.c (file:line per function below); statements are prepared with bound values
 * instead of being printed into SQL text, which stores the same values (REAL-affinity columns
 * parse the bound "%f" text exactly as they parse the reference's literals). */
#define _GNU_SOURCE /* PTHREAD_RECURSIVE_MUTEX_INITIALIZER_NP (Asterisk builds with it too) */
#include "asterisk.h"

#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <openssl/evp.h>
#include <sqlite3.h>

#include "asterisk/json.h"
#include "asterisk/logger.h"
#include "asterisk/utils.h"

#include "fp_catalog.h"

#define NULL_MICRO INT32_MIN /* TFP_NULL_MICRO */

static sqlite3* g_db = NULL;
static char g_backup[4096] = FPC_DEF_BACKUP_DATABASE;
static pthread_mutex_t g_lock = PTHREAD_RECURSIVE_MUTEX_INITIALIZER_NP;

/* init_database (fp_handler.c:673-756) with DEF_AUBIO_COEFS = 2: the same statements, in order */
static const char* const g_ddl[] = {
	"create table context_list(   name        varchar(255),   directory   varchar(1023),   primary key(name));",
	"create table audio_list(   uuid           varchar(255),   name           varchar(255),"
	"   context        varchar(255),\thash           varchar(1023));",
	"create table audio_fingerprint( context        varchar(255), audio_uuid     varchar(255),"
	" frame_idx      integer, max1 real, max2 real);",
	"create index idx_audio_fingerprint_context on audio_fingerprint(context);",
	"create index idx_audio_fingerprint_max1 on audio_fingerprint(max1);",
	"create index idx_audio_fingerprint_max2 on audio_fingerprint(max2);",
};

void fpc_set_backup_path(const char* path)
{
	pthread_mutex_lock(&g_lock);
	snprintf(g_backup, sizeof(g_backup), "%s", path ? path : FPC_DEF_BACKUP_DATABASE);
	pthread_mutex_unlock(&g_lock);
}

static bool exec_sql(const char* sql)
{
	char* err = NULL;
	if(sqlite3_exec(g_db, sql, NULL, NULL, &err) != SQLITE_OK) {
		ast_log(LOG_ERROR, "Could not execute. sql[%s], err[%s]\n", sql, err ? err : "");
		sqlite3_free(err);
		return false;
	}
	return true;
}

/* process_dml_row (db_ctx_handler.c:827-841): one backup table copied into main */
static int copy_table(void* arg, int ncols, char** values, char** columns)
{
	char* sql;
	(void)arg;
	(void)columns;
	if(ncols != 1 || values[0] == NULL) {
		return 1;
	}
	sql = sqlite3_mprintf("insert into main.%q select * from backup.%q", values[0], values[0]);
	sqlite3_exec(g_db, sql, NULL, NULL, NULL);
	sqlite3_free(sql);
	return 0;
}

bool fpc_db_init(void)
{
	size_t i;
	char* sql;

	pthread_mutex_lock(&g_lock);
	if(g_db != NULL) {
		pthread_mutex_unlock(&g_lock);
		ast_log(LOG_NOTICE, "Database is already connected.\n");
		return true;
	}
	if(sqlite3_open(":memory:", &g_db) != SQLITE_OK) { /* DEF_DATABASE_NAME, fp_handler.c:30 */
		ast_log(LOG_ERROR, "Could not initiate database. err[%s]\n", sqlite3_errmsg(g_db));
		sqlite3_close(g_db);
		g_db = NULL;
		pthread_mutex_unlock(&g_lock);
		return false;
	}
	for(i = 0; i < sizeof(g_ddl) / sizeof(g_ddl[0]); i++) {
		if(exec_sql(g_ddl[i]) == false) {
			sqlite3_close(g_db);
			g_db = NULL;
			pthread_mutex_unlock(&g_lock);
			return false;
		}
	}
	/* db_ctx_load_db_data (db_ctx_handler.c:750-772): errors are ignored as there (a missing file
	 * attaches as an empty database) */
	sql = sqlite3_mprintf("ATTACH DATABASE '%q' as backup", g_backup);
	sqlite3_exec(g_db, sql, NULL, NULL, NULL);
	sqlite3_free(sql);
	sqlite3_exec(g_db, "BEGIN", NULL, NULL, NULL);
	sqlite3_exec(g_db, "SELECT name FROM backup.sqlite_master WHERE type='table'", copy_table, NULL, NULL);
	sqlite3_exec(g_db, "COMMIT", NULL, NULL, NULL);
	sqlite3_exec(g_db, "DETACH DATABASE backup", NULL, NULL, NULL);
	pthread_mutex_unlock(&g_lock);
	return true;
}

void fpc_db_close(void)
{
	pthread_mutex_lock(&g_lock);
	if(g_db != NULL) {
		sqlite3_close(g_db);
		g_db = NULL;
	}
	pthread_mutex_unlock(&g_lock);
}

/* db_ctx_backup (db_ctx_handler.c:673-717), then db_ctx_term */
bool fpc_db_term(void)
{
	sqlite3* dst = NULL;
	sqlite3_backup* b;
	bool ok = true;
	int ret;

	pthread_mutex_lock(&g_lock);
	if(g_db == NULL) {
		pthread_mutex_unlock(&g_lock);
		return false;
	}
	if(sqlite3_open(g_backup, &dst) != SQLITE_OK) {
		ok = false;
	}
	else if((b = sqlite3_backup_init(dst, "main", g_db, "main")) == NULL) {
		ast_log(LOG_WARNING, "Could not initiate backup database.\n");
		ok = false;
	}
	else {
		while(1) {
			ret = sqlite3_backup_step(b, 5);
			if(ret == SQLITE_DONE) {
				break;
			}
			if((ret != SQLITE_OK) && (ret != SQLITE_BUSY) && (ret != SQLITE_LOCKED)) {
				ast_log(LOG_ERROR, "Could not backup the database. ret[%d]\n", ret);
				ok = false;
				break;
			}
			if((ret == SQLITE_BUSY) || (ret == SQLITE_LOCKED)) {
				sqlite3_sleep(100);
			}
		}
		sqlite3_backup_finish(b);
	}
	sqlite3_close(dst);
	sqlite3_close(g_db);
	g_db = NULL;
	pthread_mutex_unlock(&g_lock);
	return ok;
}

/* ---- rows as ast_json (db_ctx_get_record, db_ctx_handler.c:267-352) ------------------------ */

static struct ast_json* record(sqlite3_stmt* st)
{
	int i, n = sqlite3_column_count(st);
	struct ast_json* j = ast_json_object_create();
	for(i = 0; i < n; i++) {
		struct ast_json* v;
		switch(sqlite3_column_type(st, i)) {
		case SQLITE_INTEGER:
			v = ast_json_integer_create(sqlite3_column_int(st, i));
			break;
		case SQLITE_FLOAT:
			v = ast_json_real_create(sqlite3_column_double(st, i));
			break;
		case SQLITE_TEXT: {
			/* db_ctx_handler.c:311-333: text that loads as JSON keeps the loaded array / object /
			 * string, anything else is the text as a string */
			const char* t = (const char*)sqlite3_column_text(st, i);
			if(t == NULL) {
				v = ast_json_null();
				break;
			}
			v = ast_json_load_string(t, NULL);
			if(v != NULL && ast_json_typeof(v) != AST_JSON_ARRAY && ast_json_typeof(v) != AST_JSON_OBJECT &&
					ast_json_typeof(v) != AST_JSON_STRING) {
				ast_json_unref(v);
				v = NULL;
			}
			if(v == NULL) {
				v = ast_json_string_create(t);
			}
			break;
		}
		default:
			v = ast_json_null();
			break;
		}
		ast_json_object_set(j, sqlite3_column_name(st, i), v);
	}
	return j;
}

/* The first row of sql with text parameters a (and b), or NULL. */
static struct ast_json* query_one(const char* sql, const char* a, const char* b)
{
	sqlite3_stmt* st = NULL;
	struct ast_json* j = NULL;
	pthread_mutex_lock(&g_lock);
	if(g_db != NULL && sqlite3_prepare_v2(g_db, sql, -1, &st, NULL) == SQLITE_OK) {
		if(a) sqlite3_bind_text(st, 1, a, -1, SQLITE_TRANSIENT);
		if(b) sqlite3_bind_text(st, 2, b, -1, SQLITE_TRANSIENT);
		if(sqlite3_step(st) == SQLITE_ROW) {
			j = record(st);
		}
	}
	sqlite3_finalize(st);
	pthread_mutex_unlock(&g_lock);
	return j;
}

/* Every row of sql (optional text parameter a) as an array. */
static struct ast_json* query_all(const char* sql, const char* a)
{
	sqlite3_stmt* st = NULL;
	struct ast_json* arr = ast_json_array_create();
	pthread_mutex_lock(&g_lock);
	if(g_db != NULL && sqlite3_prepare_v2(g_db, sql, -1, &st, NULL) == SQLITE_OK) {
		if(a) sqlite3_bind_text(st, 1, a, -1, SQLITE_TRANSIENT);
		while(sqlite3_step(st) == SQLITE_ROW) {
			ast_json_array_append(arr, record(st));
		}
	}
	sqlite3_finalize(st);
	pthread_mutex_unlock(&g_lock);
	return arr;
}

/* One statement with up to two text parameters; false on error. */
static bool exec_bound(const char* sql, const char* a, const char* b)
{
	sqlite3_stmt* st = NULL;
	bool ok = false;
	pthread_mutex_lock(&g_lock);
	if(g_db != NULL && sqlite3_prepare_v2(g_db, sql, -1, &st, NULL) == SQLITE_OK) {
		if(a) sqlite3_bind_text(st, 1, a, -1, SQLITE_TRANSIENT);
		if(b) sqlite3_bind_text(st, 2, b, -1, SQLITE_TRANSIENT);
		ok = sqlite3_step(st) == SQLITE_DONE;
	}
	if(ok == false) {
		ast_log(LOG_WARNING, "Could not execute. sql[%s], err[%s]\n", sql, g_db ? sqlite3_errmsg(g_db) : "closed");
	}
	sqlite3_finalize(st);
	pthread_mutex_unlock(&g_lock);
	return ok;
}

/* ---- audio_list ---------------------------------------------------------------------------- */

/* create_file_hash (fp_handler.c:758-805): lower-case hex MD5 of the file's bytes */
char* fp_create_hash(const char* filename)
{
	unsigned char buf[1 << 16], md[EVP_MAX_MD_SIZE];
	unsigned int mdlen = 0, i;
	EVP_MD_CTX* ctx;
	FILE* f;
	size_t n;
	char* res;

	if(filename == NULL) {
		ast_log(LOG_WARNING, "Wrong input parameter.\n");
		return NULL;
	}
	f = fopen(filename, "rb");
	if(f == NULL) {
		ast_log(LOG_WARNING, "Could not open file. filename[%s]\n", filename);
		return NULL;
	}
	ctx = EVP_MD_CTX_new();
	if(ctx == NULL || EVP_DigestInit_ex(ctx, EVP_md5(), NULL) != 1) {
		EVP_MD_CTX_free(ctx);
		fclose(f);
		return NULL;
	}
	while((n = fread(buf, 1, sizeof(buf), f)) > 0) {
		EVP_DigestUpdate(ctx, buf, n);
	}
	fclose(f);
	EVP_DigestFinal_ex(ctx, md, &mdlen);
	EVP_MD_CTX_free(ctx);
	res = ast_malloc(2 * mdlen + 1);
	if(res == NULL) {
		return NULL;
	}
	for(i = 0; i < mdlen; i++) {
		snprintf(res + 2 * i, 3, "%02x", md[i]);
	}
	res[2 * mdlen] = '\0';
	return res;
}

/* fp_generate_uuid (fp_handler.c:1097-1109): a random (version 4) uuid, lower case, as
 * uuid_generate + uuid_unparse_lower produce with /dev/urandom */
char* fp_generate_uuid(void)
{
	unsigned char b[16];
	char* s;
	FILE* f = fopen("/dev/urandom", "rb");
	if(f == NULL || fread(b, 1, sizeof(b), f) != sizeof(b)) {
		if(f) fclose(f);
		ast_log(LOG_ERROR, "Could not read /dev/urandom.\n");
		return NULL;
	}
	fclose(f);
	b[6] = (unsigned char)((b[6] & 0x0f) | 0x40);
	b[8] = (unsigned char)((b[8] & 0x3f) | 0x80);
	s = ast_malloc(37);
	if(s == NULL) {
		return NULL;
	}
	snprintf(s, 37, "%02x%02x%02x%02x-%02x%02x-%02x%02x-%02x%02x-%02x%02x%02x%02x%02x%02x", b[0], b[1], b[2], b[3],
			b[4], b[5], b[6], b[7], b[8], b[9], b[10], b[11], b[12], b[13], b[14], b[15]);
	return s;
}

/* create_audio_list_info (fp_handler.c:479-530) */
int fpc_create_audio_list_info(const char* context, const char* filename, const char* uuid)
{
	return fpc_create_audio_list_info_ex(context, filename, uuid, NULL, 0);
}

int fpc_create_audio_list_info_ex(const char* context, const char* filename, const char* uuid, char* existing,
		size_t len)
{
	char* hash;
	const char* name;
	struct ast_json* j;
	sqlite3_stmt* st = NULL;
	int ret = -1;

	if((context == NULL) || (filename == NULL) || (uuid == NULL)) {
		ast_log(LOG_WARNING, "Wrong input parameter.\n");
		return -1;
	}
	hash = fp_create_hash(filename);
	if(hash == NULL) {
		ast_log(LOG_WARNING, "Could not create hash info.\n");
		return -1;
	}
	name = strrchr(filename, '/');
	name = name ? name + 1 : filename;
	pthread_mutex_lock(&g_lock); /* the existence check and the insert as one step */
	j = query_one("select * from audio_list where context = ? and hash = ?;", context, hash);
	if(j != NULL) {
		ast_log(LOG_VERBOSE, "The given file is already fingerprinted. context[%s], filename[%s]\n", context, filename);
		if(existing != NULL && len > 0) {
			const char* u = ast_json_string_get(ast_json_object_get(j, "uuid"));
			snprintf(existing, len, "%s", u ? u : "");
		}
		ast_json_unref(j);
		ret = 0;
	}
	else if(g_db != NULL &&
			sqlite3_prepare_v2(g_db, "insert into audio_list(uuid, name, context, hash) values (?, ?, ?, ?);", -1, &st,
					NULL) == SQLITE_OK) {
		sqlite3_bind_text(st, 1, uuid, -1, SQLITE_TRANSIENT);
		sqlite3_bind_text(st, 2, name, -1, SQLITE_TRANSIENT);
		sqlite3_bind_text(st, 3, context, -1, SQLITE_TRANSIENT);
		sqlite3_bind_text(st, 4, hash, -1, SQLITE_TRANSIENT);
		ret = sqlite3_step(st) == SQLITE_DONE ? 1 : -1;
	}
	sqlite3_finalize(st);
	pthread_mutex_unlock(&g_lock);
	if(ret < 0) {
		ast_log(LOG_ERROR, "Could not create fingerprint info.\n");
	}
	ast_free(hash);
	return ret;
}

/* get_audio_list_info (fp_handler.c:832-855) */
struct ast_json* fpc_get_audio_list_info(const char* uuid)
{
	if(uuid == NULL) {
		ast_log(LOG_WARNING, "Wrong input parameter.\n");
		return NULL;
	}
	return query_one("select * from audio_list where uuid = ?;", uuid, NULL);
}

/* fp_delete_audio_list_info's SQL (fp_handler.c:115-159) */
bool fpc_delete_audio_list_info(const char* uuid)
{
	struct ast_json* j = fpc_get_audio_list_info(uuid);
	bool ok;
	if(j == NULL) {
		ast_log(LOG_NOTICE, "Could not find audio list info.\n");
		return false;
	}
	ast_json_unref(j);
	pthread_mutex_lock(&g_lock);
	ok = exec_bound("delete from audio_list where uuid=?;", uuid, NULL);
	if(ok == false) {
		ast_log(LOG_WARNING, "Could not delete audio list info. uuid[%s]\n", uuid);
	}
	else if((ok = exec_bound("delete from audio_fingerprint where audio_uuid=?;", uuid, NULL)) == false) {
		ast_log(LOG_WARNING, "Could not delete audio fingerprint info. audio_uuid[%s]\n", uuid);
	}
	pthread_mutex_unlock(&g_lock);
	return ok;
}

struct ast_json* fp_get_audio_lists_all(void) /* fp_handler.c:414-439 */
{
	return query_all("select * from audio_list;", NULL);
}

struct ast_json* fp_get_audio_lists_by_contextname(const char* name) /* fp_handler.c:441-470 */
{
	if(name == NULL) {
		ast_log(LOG_WARNING, "Wrong input parameter.\n");
		return NULL;
	}
	return query_all("select * from audio_list where context = ?;", name);
}

/* ---- audio_fingerprint -------------------------------------------------------------------- */

/* "%f" of a stored micro-unit value (db_ctx_handler.c:479-481): the exact decimal the reference
 * printed, since the value is printf's 6-decimal rounding to begin with */
static void micro_text(int32_t m, char* out, size_t cap)
{
	const int64_t a = m < 0 ? -(int64_t)m : (int64_t)m;
	snprintf(out, cap, "%s%lld.%06lld", m < 0 ? "-" : "", (long long)(a / 1000000), (long long)(a % 1000000));
}

/* create_audio_fingerprint_info's INSERTs (fp_handler.c:559-571): one row per frame with keys
 * frame_idx, audio_uuid, max1, max2 (absent when not finite -> NULL) and context */
bool fpc_store_fingerprints(const char* context, const char* uuid, const int32_t* m1, const int32_t* m2, int64_t n)
{
	sqlite3_stmt* st = NULL;
	char t1[32], t2[32];
	int64_t i;
	bool ok = true;

	if(context == NULL || uuid == NULL || n < 0 || (n > 0 && (m1 == NULL || m2 == NULL))) {
		ast_log(LOG_WARNING, "Wrong input parameter.\n");
		return false;
	}
	pthread_mutex_lock(&g_lock);
	if(g_db == NULL || exec_sql("BEGIN") == false) {
		pthread_mutex_unlock(&g_lock);
		return false;
	}
	if(sqlite3_prepare_v2(g_db,
			"insert into audio_fingerprint(frame_idx, audio_uuid, max1, max2, context) values (?, ?, ?, ?, ?);", -1, &st,
			NULL) != SQLITE_OK) {
		ok = false;
	}
	for(i = 0; ok && i < n; i++) {
		sqlite3_bind_int64(st, 1, i);
		sqlite3_bind_text(st, 2, uuid, -1, SQLITE_STATIC);
		if(m1[i] == NULL_MICRO) {
			sqlite3_bind_null(st, 3);
		}
		else {
			micro_text(m1[i], t1, sizeof(t1));
			sqlite3_bind_text(st, 3, t1, -1, SQLITE_STATIC);
		}
		if(m2[i] == NULL_MICRO) {
			sqlite3_bind_null(st, 4);
		}
		else {
			micro_text(m2[i], t2, sizeof(t2));
			sqlite3_bind_text(st, 4, t2, -1, SQLITE_STATIC);
		}
		sqlite3_bind_text(st, 5, context, -1, SQLITE_STATIC);
		if(sqlite3_step(st) != SQLITE_DONE) {
			ast_log(LOG_WARNING, "Could not insert fingerprint data.\n");
			ok = false;
		}
		sqlite3_reset(st);
	}
	sqlite3_finalize(st);
	exec_sql(ok ? "COMMIT" : "ROLLBACK");
	pthread_mutex_unlock(&g_lock);
	return ok;
}

void fpc_rows_free(fpc_rows* r)
{
	int32_t i;
	if(r == NULL) {
		return;
	}
	for(i = 0; r->uuids && i < r->nclips; i++) {
		ast_free(r->uuids[i]);
	}
	ast_free(r->uuids);
	ast_free(r->frame_offsets);
	ast_free(r->m1);
	ast_free(r->m2);
	memset(r, 0, sizeof(*r));
}

/* A stored max value -> micro-units: the REAL is SQLite's parse of the "%f" text, so rounding
 * x * 10^6 recovers the integer exactly; NULL -> NULL_MICRO. False for a value no fingerprint
 * can hold (text, out of range). */
static bool column_micro(sqlite3_stmt* st, int i, int32_t* out)
{
	double v, m;
	switch(sqlite3_column_type(st, i)) {
	case SQLITE_NULL:
		*out = NULL_MICRO;
		return true;
	case SQLITE_INTEGER:
	case SQLITE_FLOAT:
		v = sqlite3_column_double(st, i);
		m = nearbyint(v * 1e6);
		if(!(m > (double)INT32_MIN && m <= (double)INT32_MAX)) {
			return false;
		}
		*out = (int32_t)m;
		return true;
	default:
		return false;
	}
}

bool fpc_load_fingerprints(fpc_rows* r)
{
	sqlite3_stmt* st = NULL;
	int64_t cap = 0, n = 0;
	int32_t ccap = 0;
	bool ok = true;

	memset(r, 0, sizeof(*r));
	pthread_mutex_lock(&g_lock);
	if(g_db == NULL || sqlite3_prepare_v2(g_db,
			"select audio_uuid, max1, max2 from audio_fingerprint where audio_uuid is not null"
			" order by audio_uuid, rowid;", -1, &st, NULL) != SQLITE_OK) {
		pthread_mutex_unlock(&g_lock);
		return false;
	}
	while(ok && sqlite3_step(st) == SQLITE_ROW) {
		const char* u = (const char*)sqlite3_column_text(st, 0);
		if(r->nclips == 0 || strcmp(r->uuids[r->nclips - 1], u) != 0) {
			if(r->nclips + 1 >= ccap) {
				int32_t nc = ccap ? 2 * ccap : 1024;
				char** nu = ast_realloc(r->uuids, sizeof(char*) * (size_t)nc);
				int64_t* no = nu ? ast_realloc(r->frame_offsets, sizeof(int64_t) * ((size_t)nc + 1)) : NULL;
				if(nu) r->uuids = nu;
				if(no) r->frame_offsets = no;
				if(nu == NULL || no == NULL) {
					ok = false;
					break;
				}
				ccap = nc;
			}
			r->frame_offsets[r->nclips] = n;
			r->uuids[r->nclips] = ast_strdup(u);
			r->nclips++;
		}
		if(n == cap) {
			int64_t nc = cap ? 2 * cap : 1 << 16;
			int32_t* a = ast_realloc(r->m1, sizeof(int32_t) * (size_t)nc);
			int32_t* b = a ? ast_realloc(r->m2, sizeof(int32_t) * (size_t)nc) : NULL;
			if(a) r->m1 = a;
			if(b) r->m2 = b;
			if(a == NULL || b == NULL) {
				ok = false;
				break;
			}
			cap = nc;
		}
		if(column_micro(st, 1, &r->m1[n]) == false || column_micro(st, 2, &r->m2[n]) == false) {
			ast_log(LOG_ERROR, "audio_fingerprint row of %s holds a value no fingerprint has.\n", u);
			ok = false;
			break;
		}
		n++;
	}
	sqlite3_finalize(st);
	pthread_mutex_unlock(&g_lock);
	if(ok && r->frame_offsets == NULL) {
		r->frame_offsets = ast_calloc(1, sizeof(int64_t));
		ok = r->frame_offsets != NULL;
	}
	if(ok == false) {
		fpc_rows_free(r);
		return false;
	}
	r->frame_offsets[r->nclips] = n;
	return true;
}

/* ---- context_list (fp_handler.c:912-1095) ----------------------------------------------------- */

struct ast_json* fp_get_context_lists_all(void)
{
	return query_all("select * from context_list;", NULL);
}

struct ast_json* fp_get_context_list_info(const char* name)
{
	if(name == NULL) {
		ast_log(LOG_WARNING, "Wrong input parameter.\n");
		return NULL;
	}
	return query_one("select * from context_list where name == ?;", name, NULL);
}

bool fp_create_context_list_info(const char* name, const char* directory, bool replace)
{
	if(name == NULL || directory == NULL) {
		ast_log(LOG_WARNING, "Wrong input parameter.\n");
		return false;
	}
	if(exec_bound(replace ? "insert or replace into context_list(name, directory) values (?, ?);"
	                      : "insert into context_list(name, directory) values (?, ?);", name, directory) == false) {
		ast_log(LOG_WARNING, "Could not create context list info. name[%s]\n", name);
		return false;
	}
	return true;
}

bool fp_delete_context_list_info(const char* name)
{
	struct ast_json* j;
	struct ast_json* lists;
	size_t i;

	if(name == NULL) {
		ast_log(LOG_WARNING, "Wrong input parameter.\n");
		return false;
	}
	j = fp_get_context_list_info(name);
	if(j == NULL) {
		ast_log(LOG_NOTICE, "Could not find context info. context[%s]\n", name);
		return false;
	}
	ast_json_unref(j);
	lists = fp_get_audio_lists_by_contextname(name);
	if(lists == NULL) {
		ast_log(LOG_WARNING, "Could not get audio_list info. context[%s]\n", name);
		return false;
	}
	for(i = 0; i < ast_json_array_size(lists); i++) {
		const char* uuid = ast_json_string_get(ast_json_object_get(ast_json_array_get(lists, i), "uuid"));
		if(uuid == NULL) {
			continue;
		}
		if(fp_delete_audio_list_info(uuid) != true) {
			ast_log(LOG_WARNING, "Could not delete audio_list info. uuid[%s]\n", uuid);
		}
	}
	ast_json_unref(lists);
	if(exec_bound("delete from context_list where name == ?;", name, NULL) == false) {
		ast_log(LOG_NOTICE, "Could not delete context_list info. name[%s]\n", name);
		return false;
	}
	return true;
}
