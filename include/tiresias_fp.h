/* tiresias_fp.h — C-ABI of the MI355X-native tiresias fingerprint engine.
 *
 * Drop-in boundary for the hot path of pchero/asterisk-tiresias (/root/reference):
 * the Asterisk-side C (application_handler.c, cli_handler.c, app_tiresias.c and the SQLite
 * catalog in db_ctx_handler.c) keeps working and calls these entry points from a thin
 * fp_handler.c shim. Plain C types only; memory is caller-allocated unless
 * stated; every int return is TFP_OK (0) or a negative TFP_E_* code, with the message in
 * tfp_engine_last_error(). All engine calls are thread-safe (serialised per engine).
 *
 * Reference interfaces replaced (file:line in /root/reference/src):
 *   tfp_fingerprint_pcm / _batch      create_audio_fingerprints      fp_handler.c:577-671
 *   tfp_index_add                     create_audio_fingerprint_info  fp_handler.c:538-575
 *                                     (+ the INSERT it issues        db_ctx_handler.c:413-556)
 *   tfp_index_remove                  fp_delete_audio_list_info's    fp_handler.c:146-157
 *                                     "delete from audio_fingerprint where audio_uuid=..."
 *   tfp_search / _batch / _pcm_batch  fp_search_fingerprint_info     fp_handler.c:207-408
 *                                     (declared in fp_handler.h:28-35)
 *   tfp_wav_decode / tfp_wav_read     new_aubio_source + aubio_source_do at the native rate
 *                                     fp_handler.c:37, :604, :633 (libaubio source_wavread)
 */
#ifndef TIRESIAS_FP_H
#define TIRESIAS_FP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TFP_ABI_VERSION 1
#define TFP_HOP 256              /* DEF_AUBIO_HOPSIZE, fp_handler.c:33 */
#define TFP_WIN 512              /* DEF_AUBIO_BUFSIZE, fp_handler.c:34 */
#define TFP_DEFAULT_TOLERANCE 0.001 /* DEF_SEARCH_TOLERANCE, fp_handler.c:41 */
#define TFP_NULL_MICRO INT32_MIN /* a max1/max2 value the reference stores as SQL NULL */

enum {
  TFP_OK = 0,
  TFP_E_ARG = -1,       /* bad argument (NULL pointer, bad size, coefs out of range ...) */
  TFP_E_HIP = -2,       /* HIP runtime / kernel launch failure */
  TFP_E_NOMEM = -3,     /* device or host allocation failed */
  TFP_E_NOENT = -4,     /* uuid not in the index */
  TFP_E_CAPACITY = -5,  /* caller buffer too small (needed size returned through out param) */
  TFP_E_EXISTS = -6,    /* uuid already indexed */
  TFP_E_NODEV = -7,     /* no usable gfx950 device */
  TFP_E_FORMAT = -8     /* audio the engine cannot take exactly (tfp_wav_*) or a malformed file */
};

typedef struct tfp_engine tfp_engine;
typedef struct tfp_plan tfp_plan;

/* One fingerprint row = one 256-sample hop (reference JSON row {frame_idx, audio_uuid,
 * max1, max2}, fp_handler.c:645-652). m1/m2 are the values as STORED: printf("%f") of
 * 10*log10|c| in integer micro-units (db_ctx_handler.c:479-481); TFP_NULL_MICRO where the
 * reference stores NULL. q1/q2 are the unrounded doubles the search loop reads back
 * (fp_handler.c:290,321); -inf where the key is absent. */
typedef struct tfp_frame {
  int32_t frame_idx;
  int32_t m1;
  int32_t m2;
  int32_t reserved;
  double q1;
  double q2;
} tfp_frame;

/* fp_search_fingerprint_info arguments (fp_handler.h:28-35). coefs in [1,2]; tolerance < 0
 * selects TFP_DEFAULT_TOLERANCE; freq_ignore_* <= 0 disables the filter. */
typedef struct tfp_search_params {
  int32_t coefs;
  int32_t freq_ignore_low;
  int32_t freq_ignore_high;
  int32_t reserved;
  double tolerance;
} tfp_search_params;

/* Result of one search: the reference returns NULL (found = 0) or
 * {uuid,...,frame_count,match_count} (fp_handler.c:394-404). */
typedef struct tfp_result {
  int32_t found;
  int32_t match_count;   /* count(*) of the winning audio_uuid */
  int32_t frame_count;   /* all query frames, ignored ones included */
  int32_t clip_id;       /* engine clip id of the winner, -1 if none */
  char uuid[64];         /* winning audio_uuid, NUL-terminated ("" if none) */
} tfp_result;

/* ---- engine ------------------------------------------------------------------------ */
int tfp_abi_version(void);
int tfp_device_count(int32_t* count);
int tfp_engine_create(int32_t device, tfp_engine** out);
void tfp_engine_destroy(tfp_engine* eng); /* destroy the engine's streams first */
const char* tfp_engine_last_error(const tfp_engine* eng); /* eng == NULL: this thread's last
                                                          * engine-less error (tfp_wav_*). The calling
                                                          * thread's last failure on eng, else eng's
                                                          * latest; the pointer stays valid until this
                                                          * thread's next failing call or last_error
                                                          * read on the same handle */
int64_t tfp_frame_count(int64_t nsamples); /* ceil(n / 256) */

/* ---- host buffers the engine reads in place ------------------------------------------- */
/* Pinned, device-mapped host memory for PCM (new in round 2). Samples handed to a query search
 * (tfp_search_pcm_batch, tfp_search_pcm) or a small tfp_fingerprint_* call from inside such a
 * buffer are read by the GPU where they lie: the call skips copying them into the engine's
 * staging (a 5 s query is 80 KB, several microseconds of batch-1 latency). Any other caller memory
 * works as before. Thread-safe, usable with every engine; the buffer must stay allocated until
 * the call that reads it returns. The Asterisk shim reads WAV files straight into one.
 * tfp_host_alloc: TFP_E_ARG for bytes == 0 or out == NULL, TFP_E_NOMEM when allocation fails. */
int tfp_host_alloc(size_t bytes, void** out);
void tfp_host_free(void* p); /* NULL is a no-op; p must come from tfp_host_alloc */

/* ---- audio ingest: the aubio_source step of create_audio_fingerprints ------------------ */
/* RIFF/WAVE -> mono int16 PCM at the file's native rate (fp_handler.c:37 DEF_AUBIO_SAMPLERATE 0,
 * :604, :633). Accepts integer PCM (format 1, or EXTENSIBLE with the PCM subformat), mono,
 * 16-bit (samples as stored) or 8-bit ((u - 128) << 8: aubio's (u - 128) / 128 exactly). Other
 * audio has aubio values between int16 steps (multichannel mean, 24/32-bit, float) and returns
 * TFP_E_FORMAT. A data size of 0 or past the end of the bytes takes the whole samples present.
 * pcm == NULL (cap 0) only sets *nsamples / *sample_rate; cap < samples -> TFP_E_CAPACITY with
 * *nsamples set. Host-only (no GPU); errors via tfp_engine_last_error(NULL). */
int tfp_wav_decode(const void* bytes, int64_t nbytes, int16_t* pcm, int64_t cap, int64_t* nsamples,
                   int32_t* sample_rate);
int tfp_wav_read(const char* path, int16_t* pcm, int64_t cap, int64_t* nsamples, int32_t* sample_rate);
/* RIFF/WAVE -> the fp32 mono hop values aubio_source_do produces (fp_handler.c:604, :633), for
 * every file tfp_wav_decode refuses as well: 8/16/24/32-bit integer PCM and 32/64-bit float
 * (format 3, or EXTENSIBLE), any channel count. Per sample: unsigned 8-bit (u - 128) / 128,
 * signed w-bit x / 2^(w-1) (32-bit x rounded to float first, as libsndfile's normalised read),
 * float as stored, double rounded to float; per frame the channels are summed in fp32 in channel
 * order and divided by the channel count in fp32 (aubio 0.4.5 sndfile/wavread downmix). Feed
 * the result to tfp_fingerprint_f32_batch / tfp_search_f32_batch. Same size-query, capacity and
 * error conventions as tfp_wav_decode. Host-only. */
int tfp_wav_decode_f32(const void* bytes, int64_t nbytes, float* x, int64_t cap, int64_t* nsamples,
                       int32_t* sample_rate);
int tfp_wav_read_f32(const char* path, float* x, int64_t cap, int64_t* nsamples, int32_t* sample_rate);

/* ---- fingerprinting: create_audio_fingerprints (fp_handler.c:577-671) -------------- */
/* One clip of mono int16 PCM at its native rate (DEF_AUBIO_SAMPLERATE 0, :37). */
int tfp_fingerprint_pcm(tfp_engine* eng, const int16_t* pcm, int64_t nsamples, int32_t sample_rate,
                        tfp_frame* out, int64_t cap, int64_t* nframes);
/* Many clips: offsets[nclips+1] are sample offsets into pcm; frames are concatenated in
 * clip order (clip c starts at sum of tfp_frame_count of clips < c). */
int tfp_fingerprint_batch(tfp_engine* eng, const int16_t* pcm, const int64_t* offsets, int32_t nclips,
                          int32_t sample_rate, tfp_frame* out, int64_t cap, int64_t* nframes);
/* The same over fp32 hop values (tfp_wav_decode_f32: multichannel, 24/32-bit or float audio):
 * aubio's x is taken as given instead of int16 / 32768. For int16-valued input (x = s / 32768)
 * the frames equal tfp_fingerprint_batch's on s. */
int tfp_fingerprint_f32_batch(tfp_engine* eng, const float* x, const int64_t* offsets, int32_t nclips,
                              int32_t sample_rate, tfp_frame* out, int64_t cap, int64_t* nframes);

/* Device-resident batches (inputs already in HBM; used by the benchmark and by callers that
 * keep PCM on the GPU). A plan uploads the clip layout once. d_micro receives 2 int32 per
 * frame (m1, m2), d_db 2 doubles per frame (q1, q2) or may be NULL. stream: hipStream_t or
 * NULL for the engine's stream; a NULL-stream call (here and in every device form below) is
 * ordered after the work queued on the HIP null stream before it and before the null stream's
 * later work (the null stream is torch's default stream; the engine's stream is non-blocking).
 * Asynchronous: returns after the launch. */
int tfp_plan_create(tfp_engine* eng, const int64_t* offsets, int32_t nclips, int32_t sample_rate,
                    tfp_plan** out);
void tfp_plan_destroy(tfp_plan* plan);
int64_t tfp_plan_frames(const tfp_plan* plan);
int tfp_fingerprint_device(tfp_engine* eng, const tfp_plan* plan, const int16_t* d_pcm, int32_t* d_micro,
                           double* d_db, void* stream);

/* ---- enrolled index: the audio_fingerprint table (fp_handler.c:713-753) ------------- */
/* Append one clip's rows (create_audio_fingerprint_info). m1/m2 in micro-units. */
int tfp_index_add(tfp_engine* eng, const char* uuid, const int32_t* m1, const int32_t* m2, int32_t nframes,
                  int32_t* clip_id);
/* Append nclips clips whose rows are already on the device: d_micro holds 2 int32 per frame
 * in the layout tfp_fingerprint_device writes, frame_offsets[nclips+1] on the host. */
int tfp_index_add_device(tfp_engine* eng, int32_t nclips, const char* const* uuids, const int64_t* frame_offsets,
                         const int32_t* d_micro, void* stream);
/* Append nclips clips from host rows (m1/m2 indexed by frame_offsets[0..nclips]); the bulk
 * form of tfp_index_add used to load an audio_recongition.db snapshot (fp_init ->
 * db_ctx_load_db_data, fp_handler.c:68-90, db_ctx_handler.c:750-772). All-or-nothing on
 * argument errors (bad/duplicate uuid). */
int tfp_index_add_batch(tfp_engine* eng, int32_t nclips, const char* const* uuids, const int64_t* frame_offsets,
                        const int32_t* m1, const int32_t* m2);
/* Read back one clip's stored rows in frame order (for the fp_term backup,
 * db_ctx_backup db_ctx_handler.c:673-717). *nframes always receives the row count;
 * TFP_E_CAPACITY if cap is smaller. */
int tfp_index_rows(tfp_engine* eng, const char* uuid, int32_t* m1, int32_t* m2, int64_t cap, int64_t* nframes);
int tfp_index_remove(tfp_engine* eng, const char* uuid);
int tfp_index_clear(tfp_engine* eng);
int tfp_index_stats(tfp_engine* eng, int64_t* nrows, int32_t* nclips);
/* Rebuild the sorted device index now (otherwise done lazily by the next search). After the first
 * build, adds and removals are merged into the sorted index in one pass over it (the added rows
 * alone are sorted), as the reference's INSERTs update its max1 B-tree (fp_handler.c:559-571,
 * :745-753); a full re-sort happens only for the first build, after many removals (staging
 * compaction) or when the new rows outnumber half the index. */
int tfp_index_commit(tfp_engine* eng);
/* How the index was brought up to date so far: full sorts and incremental merges (new in round 3;
 * either pointer may be NULL). */
int tfp_index_build_stats(tfp_engine* eng, int64_t* full_builds, int64_t* merges);
/* Index delta (new in round 4): up to 512 clips enrolled since the last merge are searched beside
 * the sorted index by the coefs = 1 paths (the dialplan's, application_handler.c:180) without a
 * merge: an enrolment then costs its own rows, as the reference's INSERT into its B-tree does
 * (fp_handler.c:559-571, :745-753). coefs = 2 searches (round 6) sweep the delta's own clip-set cache
 * beside the main one. The delta is merged when it outgrows that, when a clip of the sorted index is
 * removed, or before a search that reads the sorted rows (a coefs = 1 tolerance above 8, a coefs = 2
 * tolerance above 0.49, a row-scan fallback); results are unchanged either way. TFP_INDEX_DELTA=0 at engine
 * creation turns it off. Stats: delta updates so far and the clips in the delta now. */
int tfp_index_delta_stats(tfp_engine* eng, int64_t* delta_updates, int32_t* delta_clips);
/* The coefs = 2 clip-set caches (new in round 6): builds so far, searches served by a cached
 * tolerance (the active one or one of three others kept, least recently used out), builds made from
 * the clip order (tolerances up to 0.49: a filter, no sort), the clip order's full builds (one
 * radix sort per full index build, when first needed) and merges (carried through every index
 * merge), and the index delta's caches built and sweeps run over them (an enrolment followed by a
 * coefs = 2 search: the main caches stay, the delta's rows get their own). Any pointer may be NULL. */
/* The coefs = 2 sweep's frame sort per batch (new in round 6): batches whose hand-written bin sort
 * stood, batches sorted by the library sort (a first pass that could not take the bin sort, or the
 * redo), speculative passes redone (an overfull bin, a window width outside the packed key, a frame
 * for the row scan), and the crowd bins (one value: the silence floor) the bin sort copied unsorted.
 * Any pointer may be NULL. */
int tfp_sweep_stats(tfp_engine* eng, int64_t* bins, int64_t* library, int64_t* redone, int64_t* crowd_bins);
int tfp_index_cache_stats(tfp_engine* eng, int64_t* cache_builds, int64_t* cache_hits, int64_t* from_order,
                          int64_t* order_builds, int64_t* order_merges, int64_t* delta_cache_builds,
                          int64_t* delta_sweeps);
/* Multi-GPU sharding: override the tie-break key of each live clip (default: its rank among
 * this engine's uuids). keys[clip_id] must order like the uuids across all shards and be
 * distinct over live clips. A clip added after this call has no key: the next search (or
 * tfp_index_commit) fails with TFP_E_ARG until the keys are set again; nclip_ids = 0 clears
 * the override. */
int tfp_index_set_tiebreak(tfp_engine* eng, const int32_t* keys, int32_t nclip_ids);
/* The override's keys of clip ids [first_clip_id, first_clip_id + n) only (new in round 6): a device
 * group gives each clip enrolled since the last update its key without re-sending every clip's
 * (first_clip_id <= the number of keys set so far). Keys of clips added since the last index update
 * cost the next update O(new clips); keys of older clips refresh every column's. */
int tfp_index_update_tiebreak(tfp_engine* eng, int32_t first_clip_id, const int32_t* keys, int32_t n);

/* ---- search: fp_search_fingerprint_info (fp_handler.c:207-408) ---------------------- */
int tfp_search(tfp_engine* eng, const tfp_frame* frames, int32_t nframes, const tfp_search_params* params,
               tfp_result* out);
/* qoffsets[nqueries+1] index into frames. */
int tfp_search_batch(tfp_engine* eng, const tfp_frame* frames, const int64_t* qoffsets, int32_t nqueries,
                     const tfp_search_params* params, tfp_result* out);
/* PCM in, results out: fingerprints the queries on the GPU and searches without a host
 * round trip of the frames (fp_handler.c:275 + :287-374). */
int tfp_search_pcm_batch(tfp_engine* eng, const int16_t* pcm, const int64_t* offsets, int32_t nqueries,
                         int32_t sample_rate, const tfp_search_params* params, tfp_result* out);
/* The same over fp32 hop values (tfp_wav_decode_f32). */
int tfp_search_f32_batch(tfp_engine* eng, const float* x, const int64_t* offsets, int32_t nqueries,
                         int32_t sample_rate, const tfp_search_params* params, tfp_result* out);
/* Queries in separate buffers (new in round 4): query i is the nsamples[i] int16 samples at pcms[i].
 * The results equal tfp_search_pcm_batch's over the same queries laid end to end. Samples inside
 * tfp_host_alloc buffers are read in place wherever they lie (one per channel recording, say).
 *
 * Concurrent callers (new in round 4). The reference runs one fp_search_fingerprint_info per channel
 * thread (application_handler.c:180) on one shared handle (fp_handler.c:1161-1169). Calls of
 * tfp_search_pcm_batch, tfp_search_f32_batch and tfp_search_pcm_gather with at most 16 queries each
 * are coalesced: a call made while another batch runs on the engine waits for it, then runs together
 * with every other waiting call of the same sample format, rate and search parameters as one batch
 * (<= 512 queries). A lone call runs at once. Each call gets exactly its own results.
 * TFP_COALESCE=0 in the environment at engine creation turns this off. tfp_search_coalesce_stats:
 * calls taken through the coalescer and the batches they ran as (either pointer may be NULL). */
int tfp_search_pcm_gather(tfp_engine* eng, const int16_t* const* pcms, const int64_t* nsamples, int32_t nqueries,
                          int32_t sample_rate, const tfp_search_params* params, tfp_result* out);
int tfp_search_coalesce_stats(tfp_engine* eng, int64_t* calls, int64_t* batches);
/* Device form for benchmarks / sharded search: per query a 64-bit key
 * (match_count << 32 | tiebreak key), 0 = NOTFOUND, written to d_keys[nqueries] (device).
 * The maximum key over shards is the global winner (RCCL allreduce MAX). */
int tfp_search_device(tfp_engine* eng, const tfp_plan* plan, const int16_t* d_pcm,
                      const tfp_search_params* params, uint64_t* d_keys, void* stream);
/* The same from frame values already on the device: d_q holds 2 doubles per frame (q1, q2 as
 * tfp_fingerprint_device writes them to d_db), queries at frame offsets qoffsets[nqueries+1]
 * (host). Lets N ranks each fingerprint 1/N of a query batch, all-gather the frame values and
 * search their clip shard (the reference's per-frame SQL, fp_handler.c:287-374, on q1/q2). */
int tfp_search_q_device(tfp_engine* eng, const double* d_q, const int64_t* qoffsets, int32_t nqueries,
                        const tfp_search_params* params, uint64_t* d_keys, void* stream);
/* Map a tie-break key from tfp_search_device back to the uuid (this engine's clips only). */
int tfp_index_uuid_of_key(tfp_engine* eng, int32_t key, char* uuid, int32_t len);

/* ---- live channels: rolling fingerprint + match (configs[4]) --------------------------
 * The dialplan app records `duration` ms of a channel to a WAV and searches it
 * (application_handler.c:152-185, record_voice :248-312). A stream keeps the most recent
 * window_samples of every channel on the GPU; after each tick (every channel's next
 * tick_samples, SLIN 20 ms = 160 samples at 8 kHz) the result of a channel whose history
 * holds a full window equals fp_search_fingerprint_info on a recording of exactly those
 * samples. Channels with less history report found = 0, frame_count = 0. */
typedef struct tfp_stream tfp_stream;
int tfp_stream_create(tfp_engine* eng, int32_t nchannels, int32_t sample_rate, int64_t window_samples,
                      tfp_stream** out);
void tfp_stream_destroy(tfp_stream* st); /* before tfp_engine_destroy of its engine */
/* A new call on `channel` (< 0: every channel): its history restarts empty. */
int tfp_stream_reset(tfp_stream* st, int32_t channel);
/* pcm[nchannels][tick_samples] (host); tick_samples <= window_samples. params NULL: only
 * ingest. out[nchannels] receives each channel's result when params != NULL. */
int tfp_stream_push(tfp_stream* st, const int16_t* pcm, int32_t tick_samples, const tfp_search_params* params,
                    tfp_result* out);

/* ---- device groups: the node's GPUs behind one index (new in round 3) -------------------
 * The module's enrolled DB sharded over one engine per listed device (the reference
 * has one SQLite DB, fp_handler.c:30): each clip lives on one engine (the one holding the fewest
 * rows when it is added) and is never split, since the per-frame GROUP BY audio_uuid of
 * fp_handler.c:353 is not additive over a split clip. Every search runs on all engines in parallel
 * (a worker thread per engine); the engines carry the group-wide uuid ranks as tie-break keys, so
 * the per-query key (match_count << 32 | rank) of each shard combines by an integer max into the
 * reference's winner (count(*) DESC, ties to the greatest audio_uuid, fp_handler.c:367-374).
 * Batches of >= 64 equal-length int16 queries per engine are query-sharded: each engine
 * fingerprints its share and the frame values are exchanged GPU to GPU (peer copies over xGMI);
 * smaller batches and stream ticks are fingerprinted by every engine, so the latency path has no
 * exchange. A device may be listed more than once (shards sharing a GPU). Results as the engine
 * calls, except tfp_result.clip_id = the index of the engine holding the winner. Thread-safe
 * (calls are serialised per group); errors through tfp_group_last_error. */
typedef struct tfp_group tfp_group;
int tfp_group_create(const int32_t* devices, int32_t ndevices, tfp_group** out);
void tfp_group_destroy(tfp_group* g); /* destroy its streams first */
int32_t tfp_group_size(const tfp_group* g);
/* Peer access among the group's distinct devices (new in round 6): ordered pairs of distinct
 * devices, how many of them hipDeviceCanAccessPeer allows, and for how many
 * hipDeviceEnablePeerAccess succeeded (or was already on). Any pointer may be NULL. */
int tfp_group_peer_stats(const tfp_group* g, int32_t* pairs, int32_t* can_access, int32_t* enabled);
/* The group's tie-break keys (new in round 6): respaces (every key re-spread and sent to every shard:
 * the first enrolment, a large batch, a gap exhausted), pushes of new clips' keys only, and the
 * shards' index delta updates that still re-sent every main column's key. An enrolment of a few
 * clips costs a push of their keys, not a pass over every clip. Any pointer may be NULL. */
int tfp_group_tiebreak_stats(tfp_group* g, int64_t* respaces, int64_t* partial_pushes, int64_t* shard_full_key_updates);
const char* tfp_group_last_error(const tfp_group* g);
tfp_engine* tfp_group_engine(tfp_group* g, int32_t shard); /* for stats; do not change its index */
int tfp_group_fingerprint_batch(tfp_group* g, const int16_t* pcm, const int64_t* offsets, int32_t nclips,
                                int32_t sample_rate, tfp_frame* out, int64_t cap, int64_t* nframes);
int tfp_group_fingerprint_f32_batch(tfp_group* g, const float* x, const int64_t* offsets, int32_t nclips,
                                    int32_t sample_rate, tfp_frame* out, int64_t cap, int64_t* nframes);
int tfp_group_index_add(tfp_group* g, const char* uuid, const int32_t* m1, const int32_t* m2, int32_t nframes);
int tfp_group_index_add_batch(tfp_group* g, int32_t nclips, const char* const* uuids, const int64_t* frame_offsets,
                              const int32_t* m1, const int32_t* m2);
int tfp_group_index_remove(tfp_group* g, const char* uuid);
int tfp_group_index_clear(tfp_group* g);
int tfp_group_index_rows(tfp_group* g, const char* uuid, int32_t* m1, int32_t* m2, int64_t cap, int64_t* nframes);
int tfp_group_index_stats(tfp_group* g, int64_t* nrows, int32_t* nclips);
int tfp_group_index_commit(tfp_group* g);
int tfp_group_search_batch(tfp_group* g, const tfp_frame* frames, const int64_t* qoffsets, int32_t nqueries,
                           const tfp_search_params* params, tfp_result* out);
int tfp_group_search_pcm_batch(tfp_group* g, const int16_t* pcm, const int64_t* offsets, int32_t nqueries,
                               int32_t sample_rate, const tfp_search_params* params, tfp_result* out);
int tfp_group_search_f32_batch(tfp_group* g, const float* x, const int64_t* offsets, int32_t nqueries,
                               int32_t sample_rate, const tfp_search_params* params, tfp_result* out);
/* tfp_search_pcm_gather and the coalescing of concurrent calls (as for one engine) on a group: the
 * channel threads' batch-1 searches through the shim run as shared batches on every GPU. */
int tfp_group_search_pcm_gather(tfp_group* g, const int16_t* const* pcms, const int64_t* nsamples, int32_t nqueries,
                                int32_t sample_rate, const tfp_search_params* params, tfp_result* out);
int tfp_group_search_coalesce_stats(tfp_group* g, int64_t* calls, int64_t* batches);
/* Live channels on a group: every engine keeps every channel's window and matches it against its
 * clips each tick; out[nchannels] = the combined results (as tfp_stream_push). */
typedef struct tfp_group_stream tfp_group_stream;
int tfp_group_stream_create(tfp_group* g, int32_t nchannels, int32_t sample_rate, int64_t window_samples,
                            tfp_group_stream** out);
void tfp_group_stream_destroy(tfp_group_stream* st);
int tfp_group_stream_reset(tfp_group_stream* st, int32_t channel);
int tfp_group_stream_push(tfp_group_stream* st, const int16_t* pcm, int32_t tick_samples,
                          const tfp_search_params* params, tfp_result* out);

/* ---- deterministic synthetic PCM (benchmark / test data; identical host and device) -- */
/* One spec per clip: samples s of clip = synth(seed, clip, offset + s). */
typedef struct tfp_synth_spec {
  uint64_t seed;
  int64_t clip;
  int64_t offset;
} tfp_synth_spec;
int tfp_synth_pcm(const tfp_synth_spec* specs, int32_t nclips, int64_t samples_per_clip, int16_t* out);
int tfp_synth_pcm_device(tfp_engine* eng, const tfp_synth_spec* specs, int32_t nclips, int64_t samples_per_clip,
                         int16_t* d_out, void* stream);

/* ---- misc --------------------------------------------------------------------------- */
int tfp_synchronize(tfp_engine* eng, void* stream);

#ifdef __cplusplus
}
#endif
#endif
