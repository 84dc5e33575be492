/* fp_handler_tfp.c — the hot half of the reference's engine facade (src/fp_handler.h:13-38) on
 * the MI355X engines (include/tiresias_fp.h): a device group over the node's GPUs, the enrolled
 * clips sharded over them. Built into app_tiresias.so with shim/fp_catalog.c (the catalog half:
 * the reference's SQLite tables and backup) in place of the reference's fp_handler.c and
 * db_ctx_handler.c.
 *
 *   fp_init / fp_term                fp_handler.c:68-108   + the GPU engines and their index
 *   fp_craete_audio_list_info        fp_handler.c:161-197  (sic "craete": the reference's name)
 *   fp_delete_audio_list_info        fp_handler.c:115-159  + tfp_group_index_remove
 *   fp_search_fingerprint_info       fp_handler.c:207-408
 *
 * Conventions kept: false / NULL plus ast_log on errors; the search returns NULL both for
 * NOTFOUND and for errors (application_handler.c:180-191 maps both to TIRSTATUS=NOTFOUND);
 * a file already enrolled in the context is a success (fp_handler.c:181-185); the result is
 * {uuid, name, context, hash, frame_count, match_count}, owned by the caller (ast_json_unref).
 * Every tfp_group_* call is serialised per group, so the channel threads need no lock here. */
#include "asterisk.h"

#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "asterisk/json.h"
#include "asterisk/logger.h"
#include "asterisk/utils.h"

#include "fp_catalog.h"
#include "fp_handler_tfp.h"
#include "tiresias_fp.h"

static tfp_group* g_tfp = NULL; /* the module's engines: one per configured GPU (fp_set_gpu_devices) */
static char g_devices[256] = ""; /* "" : every visible GPU */
static void pcm_pool_drain(void);

/* fp_set_gpu_devices: "0,2,5", "0-7", or "" / NULL for every visible GPU (a device may repeat) */
void fp_set_gpu_devices(const char* list)
{
	snprintf(g_devices, sizeof(g_devices), "%s", list ? list : "");
}

static bool create_group(void)
{
	int32_t dev[64], n = 0, count = 0, a, b;
	const char* p = g_devices;
	char* end;

	if(tfp_device_count(&count) != TFP_OK || count <= 0) {
		return false;
	}
	while(*p != '\0' && n < 64) {
		if(*p == ',' || *p == ' ') {
			p++;
			continue;
		}
		a = (int32_t)strtol(p, &end, 10);
		if(end == p) {
			return false;
		}
		b = a;
		if(*end == '-') {
			p = end + 1;
			b = (int32_t)strtol(p, &end, 10);
			if(end == p) {
				return false;
			}
		}
		for(; a <= b && n < 64; a++) {
			dev[n++] = a;
		}
		p = end;
	}
	if(n == 0) {
		for(a = 0; a < count && a < 64; a++) {
			dev[n++] = a;
		}
	}
	return tfp_group_create(dev, n, &g_tfp) == TFP_OK;
}

bool fp_get_search_stats(int64_t* calls, int64_t* batches)
{
	return g_tfp != NULL && tfp_group_search_coalesce_stats(g_tfp, calls, batches) == TFP_OK;
}

/* fp_init (fp_handler.c:68-90): the catalog (init_database + the backup's tables), the engine, and
 * the GPU index from the restored audio_fingerprint table in one tfp_group_index_add_batch. A failure
 * closes whatever was opened, without writing the backup. */
bool fp_init(void)
{
	fpc_rows rows;

	if(fpc_db_init() == false) {
		ast_log(LOG_ERROR, "Could not initiate database.\n");
		return false;
	}
	if(create_group() == false) {
		ast_log(LOG_ERROR, "Could not create the MI355X fingerprint engines. devices[%s]\n", g_devices);
		g_tfp = NULL;
		fpc_db_close();
		return false;
	}
	if(fpc_load_fingerprints(&rows) == false) {
		ast_log(LOG_ERROR, "Could not load the database data.\n");
		tfp_group_destroy(g_tfp);
		g_tfp = NULL;
		fpc_db_close();
		return false;
	}
	if((rows.nclips > 0 && tfp_group_index_add_batch(g_tfp, rows.nclips, (const char* const*)rows.uuids,
			rows.frame_offsets, rows.m1, rows.m2) != TFP_OK) || tfp_group_index_commit(g_tfp) != TFP_OK) {
		ast_log(LOG_ERROR, "Could not load the fingerprint index: %s\n", tfp_group_last_error(g_tfp));
		fpc_rows_free(&rows);
		tfp_group_destroy(g_tfp);
		g_tfp = NULL;
		fpc_db_close();
		return false;
	}
	fpc_rows_free(&rows);
	return true;
}

/* fp_term (fp_handler.c:92-108): the backup (the rows were written to audio_fingerprint at
 * enrolment), then the engine */
bool fp_term(void)
{
	bool ret = fpc_db_term();
	pcm_pool_drain();
	tfp_group_destroy(g_tfp);
	g_tfp = NULL;
	if(ret == false) {
		ast_log(LOG_ERROR, "Could not write database.\n");
	}
	return ret;
}

/* int16 sample buffers in engine-mapped host memory (tfp_host_alloc), which the engine reads in
 * place instead of copying into its staging. Pooled: pinning memory costs more than the copy it
 * saves. The channel threads search concurrently, so the pool is locked. */
#define PCM_POOL 32
static struct {
	int16_t* p;
	int64_t cap;
} g_pool[PCM_POOL];
static int g_npool = 0;
static pthread_mutex_t g_pool_lock = PTHREAD_MUTEX_INITIALIZER;

static int16_t* pcm_get(int64_t n, int64_t* cap)
{
	int i, best = -1;
	void* p = NULL;

	pthread_mutex_lock(&g_pool_lock);
	for(i = 0; i < g_npool; i++) {
		if(g_pool[i].cap >= n && (best < 0 || g_pool[i].cap < g_pool[best].cap)) {
			best = i;
		}
	}
	if(best >= 0) {
		int16_t* q = g_pool[best].p;
		*cap = g_pool[best].cap;
		g_pool[best] = g_pool[--g_npool];
		pthread_mutex_unlock(&g_pool_lock);
		return q;
	}
	pthread_mutex_unlock(&g_pool_lock);
	*cap = n < 80000 ? 80000 : n; /* at least 10 s at 8 kHz */
	if(tfp_host_alloc(sizeof(int16_t) * (size_t)*cap, &p) != TFP_OK) {
		*cap = 0;
		return NULL;
	}
	return (int16_t*)p;
}

static void pcm_put(int16_t* p, int64_t cap)
{
	if(p == NULL) {
		return;
	}
	pthread_mutex_lock(&g_pool_lock);
	if(g_npool < PCM_POOL) {
		g_pool[g_npool].p = p;
		g_pool[g_npool].cap = cap;
		g_npool++;
		p = NULL;
	}
	pthread_mutex_unlock(&g_pool_lock);
	tfp_host_free(p); /* pool full (NULL: kept) */
}

static void pcm_pool_drain(void)
{
	pthread_mutex_lock(&g_pool_lock);
	while(g_npool > 0) {
		g_npool--;
		tfp_host_free(g_pool[g_npool].p);
	}
	pthread_mutex_unlock(&g_pool_lock);
}

/* aubio_source (fp_handler.c:37,604,633): a WAV's mono hop values at its own rate — int16 PCM for
 * 8/16-bit mono (every Asterisk recording; in a pooled pcm_get buffer of *cap samples), else
 * (TFP_E_FORMAT) the fp32 values (multichannel mean, 24/32-bit, float). Exactly one of *pcm / *x
 * is set; release with pcm_put(*pcm, *cap) and ast_free(*x). */
static int read_audio(const char* filename, int16_t** pcm, int64_t* cap, float** x, int64_t* ns, int32_t* sr)
{
	int rc;

	*pcm = NULL;
	*cap = 0;
	*x = NULL;
	rc = tfp_wav_read(filename, NULL, 0, ns, sr);
	if(rc == TFP_OK) {
		*pcm = pcm_get(*ns ? *ns : 1, cap);
		rc = *pcm ? tfp_wav_read(filename, *pcm, *cap, ns, sr) : TFP_E_NOMEM;
	}
	else if(rc == TFP_E_FORMAT && (rc = tfp_wav_read_f32(filename, NULL, 0, ns, sr)) == TFP_OK) {
		*x = ast_malloc(sizeof(float) * (*ns ? *ns : 1));
		rc = *x ? tfp_wav_read_f32(filename, *x, *ns, ns, sr) : TFP_E_NOMEM;
	}
	if(rc != TFP_OK) {
		ast_log(LOG_WARNING, "Could not read %s: %s\n", filename, tfp_engine_last_error(NULL));
		pcm_put(*pcm, *cap);
		ast_free(*x);
		*pcm = NULL;
		*x = NULL;
		return -1;
	}
	return 0;
}

/* create_audio_fingerprint_info (fp_handler.c:538-575): the file's frames on the GPU, into the
 * index and into audio_fingerprint. */
static bool create_audio_fingerprint_info(const char* context, const char* filename, const char* uuid)
{
	int16_t* pcm;
	float* x;
	int64_t cap, ns, n, i, off[2];
	int32_t sr, *m1, *m2;
	tfp_frame* rows;
	int rc;
	bool ret;

	if(read_audio(filename, &pcm, &cap, &x, &ns, &sr) != 0) {
		return false;
	}
	n = tfp_frame_count(ns);
	rows = ast_calloc(n ? n : 1, sizeof(tfp_frame));
	m1 = ast_malloc(sizeof(int32_t) * (n ? n : 1));
	m2 = ast_malloc(sizeof(int32_t) * (n ? n : 1));
	if(rows == NULL || m1 == NULL || m2 == NULL) {
		pcm_put(pcm, cap); ast_free(x); ast_free(rows); ast_free(m1); ast_free(m2);
		return false;
	}
	off[0] = 0;
	off[1] = ns;
	rc = pcm ? tfp_group_fingerprint_batch(g_tfp, pcm, off, 1, sr, rows, n, &n)
	         : tfp_group_fingerprint_f32_batch(g_tfp, x, off, 1, sr, rows, n, &n);
	pcm_put(pcm, cap);
	ast_free(x);
	if(rc != TFP_OK) {
		ast_log(LOG_ERROR, "Could not fingerprint %s: %s\n", filename, tfp_group_last_error(g_tfp));
		ast_free(rows); ast_free(m1); ast_free(m2);
		return false;
	}
	for(i = 0; i < n; i++) {
		m1[i] = rows[i].m1;
		m2[i] = rows[i].m2;
	}
	ret = fpc_store_fingerprints(context, uuid, m1, m2, n);
	if(ret == true && tfp_group_index_add(g_tfp, uuid, m1, m2, (int32_t)n) != TFP_OK) {
		ast_log(LOG_ERROR, "Could not index %s: %s\n", filename, tfp_group_last_error(g_tfp));
		ret = false;
	}
	ast_free(rows);
	ast_free(m1);
	ast_free(m2);
	return ret;
}

bool fp_delete_audio_list_info(const char* uuid)
{
	if(uuid == NULL) {
		ast_log(LOG_WARNING, "Wrong input parameter.\n");
		return false;
	}
	if(fpc_delete_audio_list_info(uuid) == false) {
		return false;
	}
	if(tfp_group_index_remove(g_tfp, uuid) != TFP_OK) {
		ast_log(LOG_NOTICE, "Audio %s was not in the GPU index.\n", uuid);
	}
	return true;
}

bool fp_craete_audio_list_info(const char* context, const char* filename)
{
	int ret;
	char* uuid;

	if((context == NULL) || (filename == NULL)) {
		ast_log(LOG_WARNING, "Wrong input parameter.\n");
		return false;
	}
	uuid = fp_generate_uuid();
	if(uuid == NULL) {
		return false;
	}
	ret = fpc_create_audio_list_info(context, filename, uuid);
	if(ret < 0) {
		ast_log(LOG_WARNING, "Could not create audio_list info. context[%s], filename[%s]\n", context, filename);
		ast_free(uuid);
		return false;
	}
	else if(ret == 0) {
		ast_log(LOG_VERBOSE, "The given audio file is already exist in the list. context[%s], filename[%s]\n",
				context, filename);
		ast_free(uuid);
		return true;
	}
	if(create_audio_fingerprint_info(context, filename, uuid) == false) {
		ast_log(LOG_NOTICE, "Could not create audio fingerprint info.\n");
		/* (the reference passes the filename here, fp_handler.c:192, so its clean-up never
		 * matches; the shim removes the row it created) */
		fpc_delete_audio_list_info(uuid);
		ast_free(uuid);
		return false;
	}
	ast_free(uuid);
	return true;
}

/* ---- batched enrolment: app_tiresias.c:365-424's directory scan onto the GPU ----------------
 * The reference calls fp_craete_audio_list_info once per file of a context's directory (scandir,
 * alphasort). fp_create_audio_list_infos takes the whole list: the catalog rows are written in
 * the same order with the same per-context MD5 dedup (a file repeated within the list counts as
 * already enrolled), and the audio of all new files is fingerprinted by one tfp_group_fingerprint_batch
 * (per sample rate and sample format, and per ENROL_BATCH_SAMPLES) and indexed by one
 * tfp_group_index_add_batch, instead of a GPU round trip per file. */
#define ENROL_GROUPS 4
#define ENROL_BATCH_SAMPLES ((int64_t)1 << 27) /* 256 MB of int16 per batch */

typedef struct {
	int32_t sr;
	bool f32;
	int n, cap;
	int* file;         /* index into the caller's list */
	char** uuid;
	int64_t* off;      /* [n + 1] sample offsets */
	int64_t scap;      /* samples allocated */
	void* x;           /* int16 PCM or fp32 hop values */
} enrol_group;

static void group_reset(enrol_group* g)
{
	int i;
	for(i = 0; i < g->n; i++) {
		ast_free(g->uuid[i]);
	}
	g->n = 0;
	if(g->off) {
		g->off[0] = 0;
	}
}

static void group_free(enrol_group* g)
{
	group_reset(g);
	ast_free(g->file);
	ast_free(g->uuid);
	ast_free(g->off);
	ast_free(g->x);
	memset(g, 0, sizeof(*g));
}

/* fingerprint, store and index one group; returns the clips enrolled */
static int group_flush(const char* context, enrol_group* g, bool* ok)
{
	int64_t nf = 0, got = 0, i;
	int c, kept = 0, done = 0;
	tfp_frame* rows = NULL;
	int32_t *m1 = NULL, *m2 = NULL;
	int64_t* foff = NULL;
	const char** uu = NULL;
	int rc;

	if(g->n == 0) {
		return 0;
	}
	for(c = 0; c < g->n; c++) {
		nf += tfp_frame_count(g->off[c + 1] - g->off[c]);
	}
	rows = ast_calloc(nf ? nf : 1, sizeof(tfp_frame));
	m1 = ast_malloc(sizeof(int32_t) * (nf ? nf : 1));
	m2 = ast_malloc(sizeof(int32_t) * (nf ? nf : 1));
	foff = ast_malloc(sizeof(int64_t) * (g->n + 1));
	uu = ast_malloc(sizeof(char*) * g->n);
	rc = TFP_E_NOMEM;
	if(rows && m1 && m2 && foff && uu) {
		rc = g->f32 ? tfp_group_fingerprint_f32_batch(g_tfp, (const float*)g->x, g->off, g->n, g->sr, rows, nf, &got)
		            : tfp_group_fingerprint_batch(g_tfp, (const int16_t*)g->x, g->off, g->n, g->sr, rows, nf, &got);
	}
	if(rc != TFP_OK) {
		ast_log(LOG_ERROR, "Could not fingerprint %d files: %s\n", g->n, tfp_group_last_error(g_tfp));
	}
	else {
		/* the audio_fingerprint rows of each clip; a clip whose rows could not be stored is dropped */
		int64_t src = 0;
		foff[0] = 0;
		for(c = 0; c < g->n; c++) {
			const int64_t n = tfp_frame_count(g->off[c + 1] - g->off[c]);
			int32_t* a = m1 + foff[kept];
			int32_t* b = m2 + foff[kept];
			for(i = 0; i < n; i++) {
				a[i] = rows[src + i].m1;
				b[i] = rows[src + i].m2;
			}
			src += n;
			if(fpc_store_fingerprints(context, g->uuid[c], a, b, n) == false) {
				ast_log(LOG_NOTICE, "Could not create audio fingerprint info.\n");
				fpc_delete_audio_list_info(g->uuid[c]);
				continue;
			}
			uu[kept] = g->uuid[c];
			foff[kept + 1] = foff[kept] + n;
			g->file[kept] = g->file[c];
			kept++;
		}
		if(tfp_group_index_add_batch(g_tfp, kept, (const char* const*)uu, foff, m1, m2) != TFP_OK) {
			ast_log(LOG_ERROR, "Could not index %d files: %s\n", kept, tfp_group_last_error(g_tfp));
			for(c = 0; c < kept; c++) {
				fpc_delete_audio_list_info(uu[c]);
			}
		}
		else {
			for(c = 0; c < kept; c++) {
				if(ok) {
					ok[g->file[c]] = true;
				}
			}
			done = kept;
		}
	}
	if(rc != TFP_OK) {
		for(c = 0; c < g->n; c++) {
			fpc_delete_audio_list_info(g->uuid[c]);
		}
	}
	ast_free(rows);
	ast_free(m1);
	ast_free(m2);
	ast_free(foff);
	ast_free(uu);
	group_reset(g);
	return done;
}

/* appends file f's audio (ns samples at rate sr) to g; false on allocation or read errors */
static bool group_add(enrol_group* g, int f, const char* filename, char* uuid, int64_t ns)
{
	const size_t ss = g->f32 ? sizeof(float) : sizeof(int16_t);
	const int64_t at = g->off[g->n];
	int64_t got = 0;
	int32_t sr = 0;
	int rc;
	if(g->n + 1 >= g->cap) {
		int nc = g->cap ? 2 * g->cap : 64;
		int* nf = ast_realloc(g->file, sizeof(int) * (size_t)nc);
		char** nu = nf ? ast_realloc(g->uuid, sizeof(char*) * (size_t)nc) : NULL;
		int64_t* no = nu ? ast_realloc(g->off, sizeof(int64_t) * ((size_t)nc + 1)) : NULL;
		if(nf) g->file = nf;
		if(nu) g->uuid = nu;
		if(no) g->off = no;
		if(no == NULL) {
			return false;
		}
		g->cap = nc;
	}
	if(at + ns + 1 > g->scap) {
		int64_t nc = g->scap ? g->scap : (int64_t)1 << 20;
		void* nx;
		while(nc < at + ns + 1) {
			nc *= 2;
		}
		nx = ast_realloc(g->x, ss * (size_t)nc);
		if(nx == NULL) {
			return false;
		}
		g->x = nx;
		g->scap = nc;
	}
	rc = g->f32 ? tfp_wav_read_f32(filename, (float*)g->x + at, ns, &got, &sr)
	            : tfp_wav_read(filename, (int16_t*)g->x + at, ns, &got, &sr);
	if(rc != TFP_OK || got != ns || sr != g->sr) {
		return false;
	}
	g->file[g->n] = f;
	g->uuid[g->n] = uuid;
	g->off[g->n + 1] = at + ns;
	g->n++;
	return true;
}

int fp_create_audio_list_infos(const char* context, const char* const* filenames, int count, bool* ok)
{
	enrol_group groups[ENROL_GROUPS];
	int i, k, enrolled = 0;
	/* a file repeated within the list: its first copy's uuid (created in this call) and index;
	 * the repeat reports the first copy's final result, known only after the flushes */
	char** made = NULL;
	int* dup_of = NULL;
	bool* res = NULL;

	if((context == NULL) || (filenames == NULL) || (count < 0)) {
		ast_log(LOG_WARNING, "Wrong input parameter.\n");
		return -1;
	}
	made = ast_calloc(count ? count : 1, sizeof(char*));
	dup_of = ast_calloc(count ? count : 1, sizeof(int));
	res = ast_calloc(count ? count : 1, sizeof(bool));
	if(made == NULL || dup_of == NULL || res == NULL) {
		ast_free(made);
		ast_free(dup_of);
		ast_free(res);
		return -1;
	}
	for(i = 0; i < count; i++) {
		dup_of[i] = -1;
	}
	memset(groups, 0, sizeof(groups));
	for(i = 0; i < count; i++) {
		const char* f = filenames[i];
		char* uuid;
		int ret;
		int64_t ns = 0;
		int32_t sr = 0;
		bool f32 = false;
		enrol_group* g = NULL;

		char existing[64] = "";

		if(f == NULL) {
			continue;
		}
		uuid = fp_generate_uuid();
		if(uuid == NULL) {
			continue;
		}
		ret = fpc_create_audio_list_info_ex(context, f, uuid, existing, sizeof(existing));
		if(ret < 0) {
			ast_log(LOG_WARNING, "Could not create audio_list info. context[%s], filename[%s]\n", context, f);
			ast_free(uuid);
			continue;
		}
		if(ret == 0) {
			ast_log(LOG_VERBOSE, "The given audio file is already exist in the list. context[%s], filename[%s]\n",
					context, f);
			ast_free(uuid);
			res[i] = true;
			for(k = 0; k < i; k++) {
				if(made[k] != NULL && strcmp(made[k], existing) == 0) {
					dup_of[i] = k;
					break;
				}
			}
			continue;
		}
		made[i] = ast_malloc(strlen(uuid) + 1);
		if(made[i] != NULL) {
			memcpy(made[i], uuid, strlen(uuid) + 1);
		}
		/* aubio_source at the native rate: int16 PCM, else the fp32 hop values (read_audio) */
		if(tfp_wav_read(f, NULL, 0, &ns, &sr) != TFP_OK) {
			f32 = true;
			if(tfp_wav_read_f32(f, NULL, 0, &ns, &sr) != TFP_OK) {
				ast_log(LOG_WARNING, "Could not read %s: %s\n", f, tfp_engine_last_error(NULL));
				ast_log(LOG_NOTICE, "Could not create audio fingerprint info.\n");
				fpc_delete_audio_list_info(uuid);
				ast_free(uuid);
				continue;
			}
		}
		for(k = 0; k < ENROL_GROUPS; k++) {
			if(groups[k].off != NULL && groups[k].sr == sr && groups[k].f32 == f32) {
				g = &groups[k];
				break;
			}
		}
		if(g == NULL) {
			for(k = 0; k < ENROL_GROUPS && groups[k].off != NULL; k++) {
			}
			if(k == ENROL_GROUPS) { /* many formats in one scan: flush them all */
				for(k = 0; k < ENROL_GROUPS; k++) {
					enrolled += group_flush(context, &groups[k], res);
					group_free(&groups[k]);
				}
				k = 0;
			}
			g = &groups[k];
			g->sr = sr;
			g->f32 = f32;
			g->off = ast_calloc(1, sizeof(int64_t));
			if(g->off == NULL) {
				fpc_delete_audio_list_info(uuid);
				ast_free(uuid);
				continue;
			}
		}
		if(g->n > 0 && g->off[g->n] + ns > ENROL_BATCH_SAMPLES) {
			enrolled += group_flush(context, g, res);
		}
		if(group_add(g, i, f, uuid, ns) == false) {
			ast_log(LOG_WARNING, "Could not read %s: %s\n", f, tfp_engine_last_error(NULL));
			fpc_delete_audio_list_info(uuid);
			ast_free(uuid);
		}
	}
	for(k = 0; k < ENROL_GROUPS; k++) {
		enrolled += group_flush(context, &groups[k], res);
		group_free(&groups[k]);
	}
	for(i = 0; i < count; i++) {
		if(dup_of[i] >= 0) {
			res[i] = res[dup_of[i]];
		}
		if(ok) {
			ok[i] = res[i];
		}
		ast_free(made[i]);
	}
	ast_free(made);
	ast_free(dup_of);
	ast_free(res);
	return enrolled;
}

/* fp_handler.c:386-407: the winner's audio_list row + frame_count + match_count; NULL for NOTFOUND */
static struct ast_json* search_result(const tfp_result* r)
{
	struct ast_json* j_res;

	if(r->found == 0) {
		return NULL; /* no row in the temp table: NOTFOUND (fp_handler.c:367-382) */
	}
	j_res = fpc_get_audio_list_info(r->uuid); /* fp_handler.c:394-401 */
	if(j_res == NULL) {
		ast_log(LOG_ERROR, "Could not get audio list info. uuid[%s]\n", r->uuid);
		return NULL;
	}
	ast_json_object_set(j_res, "frame_count", ast_json_integer_create(r->frame_count));
	ast_json_object_set(j_res, "match_count", ast_json_integer_create(r->match_count));
	return j_res;
}

static bool search_params(tfp_search_params* p, const char* context, const int coefs, const double tolerance,
		const int freq_ignore_low, const int freq_ignore_high)
{
	if(context == NULL) {
		ast_log(LOG_WARNING, "Wrong input parameter.\n");
		return false;
	}
	if((coefs < 1) || (coefs > 2)) { /* fp_handler.c:247-250 */
		ast_log(LOG_WARNING, "Wrong coefs count. coefs[%d]\n", coefs);
		return false;
	}
	memset(p, 0, sizeof(*p));
	p->coefs = coefs;
	p->tolerance = tolerance; /* < 0: the default 0.001 (fp_handler.c:252-256) */
	p->freq_ignore_low = freq_ignore_low;
	p->freq_ignore_high = freq_ignore_high;
	return true;
}

struct ast_json* fp_search_fingerprint_info(const char* context, const char* filename, const int coefs,
		const double tolerance, const int freq_ignore_low, const int freq_ignore_high)
{
	int16_t* pcm;
	float* x;
	int64_t cap, ns, off[2];
	int32_t sr;
	int rc;
	tfp_search_params p;
	tfp_result r;

	if(filename == NULL) {
		ast_log(LOG_WARNING, "Wrong input parameter.\n");
		return NULL;
	}
	if(search_params(&p, context, coefs, tolerance, freq_ignore_low, freq_ignore_high) == false) {
		return NULL;
	}
	if(read_audio(filename, &pcm, &cap, &x, &ns, &sr) != 0) {
		return NULL;
	}
	off[0] = 0;
	off[1] = ns;
	/* concurrent channel threads' calls run as shared GPU batches (tfp_group's coalescer) */
	rc = pcm ? tfp_group_search_pcm_batch(g_tfp, pcm, off, 1, sr, &p, &r)
	         : tfp_group_search_f32_batch(g_tfp, x, off, 1, sr, &p, &r);
	pcm_put(pcm, cap);
	ast_free(x);
	if(rc != TFP_OK) {
		ast_log(LOG_ERROR, "Could not search %s: %s\n", filename, tfp_group_last_error(g_tfp));
		return NULL;
	}
	return search_result(&r);
}

/* ---- live channels: the dialplan application's recording without the /tmp WAV -------------
 * application_handler.c:152-185 records `duration` ms of the channel's voice frames
 * (record_voice, :248-312) into /tmp/tiresias-UUID.wav and searches that file. A channel keeps the
 * same samples in engine-mapped host memory instead: every voice frame is pushed as it is read,
 * and the search reads the recording in place (tfp_group_search_pcm_gather, coalesced with the
 * other channels' searches). The ring keeps the last max_ms of audio (written twice, so the kept
 * samples are always one contiguous run); with max_ms >= the recording's length it holds exactly
 * what record_voice would have written. */
struct fp_channel {
	int32_t sr;
	int64_t cap;   /* samples kept */
	int64_t n;     /* samples pushed since open / reset */
	int64_t pos;   /* ring position of the next sample */
	int16_t* ring; /* 2 * cap samples, tfp_host_alloc */
};

fp_channel* fp_channel_open(int sample_rate, int max_ms)
{
	fp_channel* ch;
	void* p = NULL;

	if(sample_rate <= 0 || max_ms <= 0) {
		ast_log(LOG_WARNING, "Wrong input parameter.\n");
		return NULL;
	}
	ch = ast_calloc(1, sizeof(*ch));
	if(ch == NULL) {
		return NULL;
	}
	ch->sr = sample_rate;
	ch->cap = ((int64_t)sample_rate * max_ms + 999) / 1000;
	if(tfp_host_alloc(sizeof(int16_t) * 2 * (size_t)ch->cap, &p) != TFP_OK) {
		ast_free(ch);
		return NULL;
	}
	ch->ring = (int16_t*)p;
	return ch;
}

bool fp_channel_push(fp_channel* ch, const int16_t* slin, int nsamples)
{
	int64_t i;

	if(ch == NULL || nsamples < 0 || (nsamples > 0 && slin == NULL)) {
		return false;
	}
	for(i = 0; i < nsamples; i++) {
		ch->ring[ch->pos] = slin[i];
		ch->ring[ch->pos + ch->cap] = slin[i];
		if(++ch->pos == ch->cap) {
			ch->pos = 0;
		}
	}
	ch->n += nsamples;
	return true;
}

void fp_channel_reset(fp_channel* ch)
{
	if(ch != NULL) {
		ch->n = 0;
		ch->pos = 0;
	}
}

struct ast_json* fp_channel_search(fp_channel* ch, const char* context, const int coefs, const double tolerance,
		const int freq_ignore_low, const int freq_ignore_high)
{
	tfp_search_params p;
	tfp_result r;
	const int16_t* q;
	int64_t len;
	int rc;

	if(ch == NULL) {
		ast_log(LOG_WARNING, "Wrong input parameter.\n");
		return NULL;
	}
	if(search_params(&p, context, coefs, tolerance, freq_ignore_low, freq_ignore_high) == false) {
		return NULL;
	}
	/* the kept samples: [0, n) before the ring wraps, else the cap samples from pos */
	len = ch->n < ch->cap ? ch->n : ch->cap;
	q = ch->n < ch->cap ? ch->ring : ch->ring + ch->pos;
	rc = tfp_group_search_pcm_gather(g_tfp, &q, &len, 1, ch->sr, &p, &r);
	if(rc != TFP_OK) {
		ast_log(LOG_ERROR, "Could not search the channel's recording: %s\n", tfp_group_last_error(g_tfp));
		return NULL;
	}
	return search_result(&r);
}

void fp_channel_close(fp_channel* ch)
{
	if(ch != NULL) {
		tfp_host_free(ch->ring);
		ast_free(ch);
	}
}
