/* fp_handler_tfp.c — the hot half of the reference's engine facade (src/fp_handler.h:13-38) on
 * the MI355X engine (include/tiresias_fp.h). Built into app_tiresias.so in place of the
 * reference's create/search code; the catalog half stays (shim/fp_catalog.h).
 *
 *   fp_init / fp_term                fp_handler.c:68-108   + the GPU engine and its index
 *   fp_craete_audio_list_info        fp_handler.c:161-197  (sic "craete": the reference's name)
 *   fp_delete_audio_list_info        fp_handler.c:115-159  + tfp_index_remove
 *   fp_search_fingerprint_info       fp_handler.c:207-408
 *
 * Conventions kept: false / NULL plus ast_log on errors; the search returns NULL both for
 * NOTFOUND and for errors (application_handler.c:180-191 maps both to TIRSTATUS=NOTFOUND);
 * a file already enrolled in the context is a success (fp_handler.c:181-185); the result is
 * {uuid, name, context, hash, frame_count, match_count}, owned by the caller (ast_json_unref).
 * Every tfp_* call is serialised per engine, so the channel threads need no lock here. */
#include "asterisk.h"

#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "asterisk/json.h"
#include "asterisk/logger.h"
#include "asterisk/utils.h"

#include "fp_catalog.h"
#include "tiresias_fp.h"

static tfp_engine* g_tfp = NULL; /* one engine (GPU 0) for the module */
static void pcm_pool_drain(void);

static bool load_clip(void* arg, const char* uuid, const int32_t* m1, const int32_t* m2, int64_t n)
{
	(void)arg;
	if(tfp_index_add(g_tfp, uuid, m1, m2, (int32_t)n, NULL) != TFP_OK) {
		ast_log(LOG_WARNING, "Could not index audio %s: %s\n", uuid, tfp_engine_last_error(g_tfp));
	}
	return true;
}

bool fp_init(void)
{
	if(fpc_db_init() == false) {
		ast_log(LOG_ERROR, "Could not initiate database.\n");
		return false;
	}
	if(tfp_engine_create(0, &g_tfp) != TFP_OK) {
		ast_log(LOG_ERROR, "Could not create the MI355X fingerprint engine.\n");
		return false;
	}
	/* the GPU index from the restored audio_fingerprint table */
	if(fpc_for_each_fingerprint_clip(load_clip, NULL) == false || tfp_index_commit(g_tfp) != TFP_OK) {
		ast_log(LOG_ERROR, "Could not load the fingerprint index: %s\n", tfp_engine_last_error(g_tfp));
		tfp_engine_destroy(g_tfp);
		g_tfp = NULL;
		return false;
	}
	return true;
}

bool fp_term(void)
{
	bool ret = fpc_db_term(); /* the rows were written to audio_fingerprint at enrolment */
	pcm_pool_drain();
	tfp_engine_destroy(g_tfp);
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
	rc = pcm ? tfp_fingerprint_pcm(g_tfp, pcm, ns, sr, rows, n, &n)
	         : tfp_fingerprint_f32_batch(g_tfp, x, off, 1, sr, rows, n, &n);
	pcm_put(pcm, cap);
	ast_free(x);
	if(rc != TFP_OK) {
		ast_log(LOG_ERROR, "Could not fingerprint %s: %s\n", filename, tfp_engine_last_error(g_tfp));
		ast_free(rows); ast_free(m1); ast_free(m2);
		return false;
	}
	for(i = 0; i < n; i++) {
		m1[i] = rows[i].m1;
		m2[i] = rows[i].m2;
	}
	ret = fpc_store_fingerprints(context, uuid, m1, m2, n);
	if(ret == true && tfp_index_add(g_tfp, uuid, m1, m2, (int32_t)n, NULL) != TFP_OK) {
		ast_log(LOG_ERROR, "Could not index %s: %s\n", filename, tfp_engine_last_error(g_tfp));
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
	if(tfp_index_remove(g_tfp, uuid) != TFP_OK) {
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
	struct ast_json* j_res;

	if((context == NULL) || (filename == NULL)) {
		ast_log(LOG_WARNING, "Wrong input parameter.\n");
		return NULL;
	}
	if((coefs < 1) || (coefs > 2)) { /* fp_handler.c:247-250 */
		ast_log(LOG_WARNING, "Wrong coefs count. coefs[%d]\n", coefs);
		return NULL;
	}
	if(read_audio(filename, &pcm, &cap, &x, &ns, &sr) != 0) {
		return NULL;
	}
	memset(&p, 0, sizeof(p));
	p.coefs = coefs;
	p.tolerance = tolerance; /* < 0: the default 0.001 (fp_handler.c:252-256) */
	p.freq_ignore_low = freq_ignore_low;
	p.freq_ignore_high = freq_ignore_high;
	off[0] = 0;
	off[1] = ns;
	rc = pcm ? tfp_search_pcm_batch(g_tfp, pcm, off, 1, sr, &p, &r)
	         : tfp_search_f32_batch(g_tfp, x, off, 1, sr, &p, &r);
	pcm_put(pcm, cap);
	ast_free(x);
	if(rc != TFP_OK) {
		ast_log(LOG_ERROR, "Could not search %s: %s\n", filename, tfp_engine_last_error(g_tfp));
		return NULL;
	}
	if(r.found == 0) {
		return NULL; /* no row in the temp table: NOTFOUND (fp_handler.c:367-382) */
	}
	j_res = fpc_get_audio_list_info(r.uuid); /* fp_handler.c:394-401 */
	if(j_res == NULL) {
		ast_log(LOG_ERROR, "Could not get audio list info. uuid[%s]\n", r.uuid);
		return NULL;
	}
	ast_json_object_set(j_res, "frame_count", ast_json_integer_create(r.frame_count));
	ast_json_object_set(j_res, "match_count", ast_json_integer_create(r.match_count));
	return j_res;
}
