/* fp_handler_tfp.h — the engine facade of the module (src/fp_handler.h:13-38, unchanged
 * signatures) as built from shim/fp_handler_tfp.c (hot half) + shim/fp_catalog.c (catalog half),
 * plus what the MI355X engine adds for the module's callers. */
#ifndef FP_HANDLER_TFP_H
#define FP_HANDLER_TFP_H

#include <stdbool.h>
#include <stdint.h>

struct ast_json;

/* src/fp_handler.h:13-38 */
bool fp_init(void);
bool fp_term(void);
bool fp_create_context_list_info(const char* name, const char* directory, bool replace);
bool fp_delete_context_list_info(const char* name);
struct ast_json* fp_get_context_lists_all(void);
struct ast_json* fp_get_context_list_info(const char* name);
struct ast_json* fp_get_audio_lists_all(void);
struct ast_json* fp_get_audio_lists_by_contextname(const char* name);
bool fp_craete_audio_list_info(const char* context, const char* filename);
bool fp_delete_audio_list_info(const char* uuid);
struct ast_json* fp_search_fingerprint_info(const char* context, const char* filename, const int coefs,
		const double tolerance, const int freq_ignore_low, const int freq_ignore_high);
char* fp_generate_uuid(void);
char* fp_create_hash(const char* filename);

/* New: fp_craete_audio_list_info over a list of files of one context, as app_tiresias.c's
 * create_new_audio_info (:365-424) calls it file by file for its directory scan. ok[i] (ok may be
 * NULL) receives what fp_craete_audio_list_info(context, filenames[i]) would return. Returns the
 * number of files newly enrolled, or -1 for bad arguments. */
int fp_create_audio_list_infos(const char* context, const char* const* filenames, int count, bool* ok);

/* New: the GPUs the module's engines run on (tfp_group: the enrolled clips sharded over them,
 * every search on all of them), before fp_init — e.g. from a "devices" option of tiresias.conf:
 * "0-7", "0,2,5", or "" / NULL for every visible GPU (the default). */
void fp_set_gpu_devices(const char* list);

/* New: how the channel threads' fp_search_fingerprint_info calls ran. Concurrent calls are
 * coalesced into shared GPU batches (tfp_group_search_pcm_batch, include/tiresias_fp.h): *calls
 * searches went through the coalescer as *batches batches. false before fp_init. */
bool fp_get_search_stats(int64_t* calls, int64_t* batches);

/* New: a live channel, for the dialplan application's record loop (application_handler.c:152-185,
 * record_voice :248-312) without the /tmp WAV round trip. Open one per call with max_ms >= the
 * recording's duration, push every voice frame's SLIN samples as it is read (160 per 20 ms frame
 * at 8 kHz), then fp_channel_search: the same result as fp_search_fingerprint_info on a WAV of
 * the samples pushed since open / reset (of the last max_ms of them, if more were pushed). The
 * samples stay in engine-mapped memory, read by the GPU in place; concurrent channels' searches run
 * as shared batches. A channel is used by one thread at a time. */
typedef struct fp_channel fp_channel;
fp_channel* fp_channel_open(int sample_rate, int max_ms);
bool fp_channel_push(fp_channel* ch, const int16_t* slin, int nsamples);
void fp_channel_reset(fp_channel* ch);
struct ast_json* fp_channel_search(fp_channel* ch, const char* context, const int coefs, const double tolerance,
		const int freq_ignore_low, const int freq_ignore_high);
void fp_channel_close(fp_channel* ch);

#endif
