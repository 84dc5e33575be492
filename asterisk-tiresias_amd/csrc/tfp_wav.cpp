// Audio ingest in front of create_audio_fingerprints: RIFF/WAVE -> the int16 samples the
// fingerprint path reads, with aubio_source semantics at the file's native rate
// (/root/reference/src/fp_handler.c:37 DEF_AUBIO_SAMPLERATE 0, :604 new_aubio_source, :633
// aubio_source_do). Host code only: the decoded PCM is what tfp_fingerprint_pcm /
// tfp_search_pcm_batch take.
//
// aubio turns a w-bit integer sample x into the fp32 value x / 2^(w-1) (8-bit data is unsigned
// and is offset by -128 first), and averages channels to mono. The engine reads int16 and
// computes x / 32768 exactly, so it accepts exactly the inputs whose aubio value is an int16
// over 32768:
//   * 16-bit mono: the stored samples;
//   * 8-bit mono: (u - 128) << 8, since (u - 128) / 128 == ((u - 128) << 8) / 32768.
// Multichannel (the mean of C channels), 24/32-bit and float data have aubio values between
// int16 steps, so tfp_wav_decode refuses them with TFP_E_FORMAT rather than silently rounding;
// tfp_wav_decode_f32 decodes them (and everything else) to the fp32 values aubio computes, for
// the fp32-sample entry points. Asterisk's own recordings (format_wav: PCM, mono, 16-bit, 8 kHz;
// application_handler.c:155) and the SLIN stream take the int16 path.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "tiresias_fp.h"

namespace {

thread_local std::string g_err;  // engine-less calls report through tfp_engine_last_error(NULL)

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

uint32_t le32(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }
uint16_t le16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }

constexpr uint16_t kFormatPcm = 1;
constexpr uint16_t kFormatFloat = 3;
constexpr uint16_t kFormatExtensible = 0xFFFE;

int read_file(const char* path, std::vector<uint8_t>& buf) {
  if (!path) return fail(TFP_E_ARG, "bad argument");
  FILE* fp = std::fopen(path, "rb");
  if (!fp) return fail(TFP_E_NOENT, std::string("cannot open ") + path);
  uint8_t chunk[1 << 16];
  size_t got;
  while ((got = std::fread(chunk, 1, sizeof chunk, fp)) > 0) buf.insert(buf.end(), chunk, chunk + got);
  const bool err = std::ferror(fp) != 0;
  std::fclose(fp);
  if (err) return fail(TFP_E_NOENT, std::string("read error on ") + path);
  if (buf.empty()) return fail(TFP_E_FORMAT, std::string("empty file ") + path);
  return TFP_OK;
}

struct WavFormat {
  uint16_t tag = 0, channels = 0, block_align = 0, bits = 0;
  uint32_t rate = 0;
};

}  // namespace

// tfp_engine_last_error(NULL) (tfp_engine.cpp) reads this; not part of the C-ABI.
extern "C" __attribute__((visibility("hidden"))) const char* tfp_ingest_last_error() { return g_err.c_str(); }

extern "C" int tfp_wav_decode(const void* bytes, int64_t nbytes, int16_t* pcm, int64_t cap, int64_t* nsamples,
                              int32_t* sample_rate) {
  if (!bytes || nbytes < 0 || !nsamples || cap < 0 || (cap > 0 && !pcm)) return fail(TFP_E_ARG, "bad argument");
  const uint8_t* b = static_cast<const uint8_t*>(bytes);
  const uint64_t n = (uint64_t)nbytes;
  if (n < 12 || std::memcmp(b, "RIFF", 4) != 0 || std::memcmp(b + 8, "WAVE", 4) != 0)
    return fail(TFP_E_FORMAT, "not a RIFF/WAVE file");
  WavFormat f;
  bool have_fmt = false;
  uint64_t pos = 12;
  while (pos + 8 <= n) {
    const uint8_t* id = b + pos;
    uint64_t size = le32(b + pos + 4);
    uint64_t body = pos + 8;
    if (std::memcmp(id, "fmt ", 4) == 0) {
      if (size < 16 || body + 16 > n) return fail(TFP_E_FORMAT, "short fmt chunk");
      f.tag = le16(b + body);
      f.channels = le16(b + body + 2);
      f.rate = le32(b + body + 4);
      f.block_align = le16(b + body + 12);
      f.bits = le16(b + body + 14);
      if (f.tag == kFormatExtensible) {
        // WAVEFORMATEXTENSIBLE: cbSize(2) validBits(2) channelMask(4) SubFormat GUID(16); the
        // GUID's first two bytes are the plain format tag.
        if (size < 40 || body + 40 > n) return fail(TFP_E_FORMAT, "short WAVE_FORMAT_EXTENSIBLE chunk");
        f.tag = le16(b + body + 24);
      }
      have_fmt = true;
    } else if (std::memcmp(id, "data", 4) == 0) {
      if (!have_fmt) return fail(TFP_E_FORMAT, "data chunk before fmt chunk");
      if (f.tag != kFormatPcm) return fail(TFP_E_FORMAT, "format tag " + std::to_string(f.tag) + " is not integer PCM");
      if (f.channels != 1)
        return fail(TFP_E_FORMAT, std::to_string(f.channels) +
                                      " channels: aubio's channel mean is not an int16 sample (mono only)");
      if (f.bits != 16 && f.bits != 8)
        return fail(TFP_E_FORMAT, std::to_string(f.bits) + "-bit samples: only 8- and 16-bit PCM map exactly to int16");
      if (f.rate == 0 || f.rate > (uint32_t)INT32_MAX) return fail(TFP_E_FORMAT, "bad sample rate");
      const uint32_t width = f.bits / 8;
      if (f.block_align != width) return fail(TFP_E_FORMAT, "block align does not match mono " + std::to_string(f.bits) + "-bit");
      // A writer that never patched the header (0 or 0xFFFFFFFF) or a truncated file: take the
      // whole samples that are present, as a streaming reader does.
      uint64_t avail = n - body;
      if (size == 0 || size > avail) size = avail;
      const int64_t ns = (int64_t)(size / width);
      *nsamples = ns;
      if (sample_rate) *sample_rate = (int32_t)f.rate;
      if (!pcm) return TFP_OK;  // size query
      if (cap < ns) return fail(TFP_E_CAPACITY, "pcm buffer holds " + std::to_string(cap) + " of " + std::to_string(ns) + " samples");
      const uint8_t* d = b + body;
      if (width == 2) {
        for (int64_t i = 0; i < ns; ++i) pcm[i] = (int16_t)le16(d + 2 * i);
      } else {
        for (int64_t i = 0; i < ns; ++i) pcm[i] = (int16_t)(((int)d[i] - 128) * 256);
      }
      return TFP_OK;
    }
    pos = body + size + (size & 1);  // RIFF chunks are padded to even sizes
  }
  return fail(TFP_E_FORMAT, have_fmt ? "no data chunk" : "no fmt chunk");
}

// fp32 form: every PCM width and float data, any channel count, as aubio 0.4.5's sndfile and
// wavread sources compute the mono hop (aubio_source_do with its default downmix): each sample
// to fp32 (unsigned 8-bit (u - 128) / 128, w-bit signed x / 2^(w-1) with 32-bit x first rounded
// to float as libsndfile's normalised read does, float data as stored, double data rounded to
// float), then per frame the channels summed in fp32 in channel order and divided by the
// channel count in fp32.
extern "C" int tfp_wav_decode_f32(const void* bytes, int64_t nbytes, float* x, int64_t cap, int64_t* nsamples,
                                  int32_t* sample_rate) {
  if (!bytes || nbytes < 0 || !nsamples || cap < 0 || (cap > 0 && !x)) return fail(TFP_E_ARG, "bad argument");
  const uint8_t* b = static_cast<const uint8_t*>(bytes);
  const uint64_t n = (uint64_t)nbytes;
  if (n < 12 || std::memcmp(b, "RIFF", 4) != 0 || std::memcmp(b + 8, "WAVE", 4) != 0)
    return fail(TFP_E_FORMAT, "not a RIFF/WAVE file");
  WavFormat f;
  bool have_fmt = false;
  uint64_t pos = 12;
  while (pos + 8 <= n) {
    const uint8_t* id = b + pos;
    uint64_t size = le32(b + pos + 4);
    const uint64_t body = pos + 8;
    if (std::memcmp(id, "fmt ", 4) == 0) {
      if (size < 16 || body + 16 > n) return fail(TFP_E_FORMAT, "short fmt chunk");
      f.tag = le16(b + body);
      f.channels = le16(b + body + 2);
      f.rate = le32(b + body + 4);
      f.block_align = le16(b + body + 12);
      f.bits = le16(b + body + 14);
      if (f.tag == kFormatExtensible) {
        if (size < 40 || body + 40 > n) return fail(TFP_E_FORMAT, "short WAVE_FORMAT_EXTENSIBLE chunk");
        f.tag = le16(b + body + 24);
      }
      have_fmt = true;
    } else if (std::memcmp(id, "data", 4) == 0) {
      if (!have_fmt) return fail(TFP_E_FORMAT, "data chunk before fmt chunk");
      const bool pcm = f.tag == kFormatPcm && (f.bits == 8 || f.bits == 16 || f.bits == 24 || f.bits == 32);
      const bool flt = f.tag == kFormatFloat && (f.bits == 32 || f.bits == 64);
      if (!pcm && !flt)
        return fail(TFP_E_FORMAT, "format tag " + std::to_string(f.tag) + " with " + std::to_string(f.bits) +
                                      "-bit samples is neither 8/16/24/32-bit PCM nor 32/64-bit float");
      if (f.channels == 0) return fail(TFP_E_FORMAT, "zero channels");
      if (f.rate == 0 || f.rate > (uint32_t)INT32_MAX) return fail(TFP_E_FORMAT, "bad sample rate");
      const uint32_t width = f.bits / 8;
      if (f.block_align != width * f.channels) return fail(TFP_E_FORMAT, "block align does not match the format");
      uint64_t avail = n - body;
      if (size == 0 || size > avail) size = avail;
      const int64_t ns = (int64_t)(size / f.block_align);
      *nsamples = ns;
      if (sample_rate) *sample_rate = (int32_t)f.rate;
      if (!x) return TFP_OK;  // size query
      if (cap < ns) return fail(TFP_E_CAPACITY, "sample buffer holds " + std::to_string(cap) + " of " + std::to_string(ns) + " samples");
      const uint8_t* d = b + body;
      const float nch = (float)f.channels;
      for (int64_t i = 0; i < ns; ++i) {
        float acc = 0.f;
        for (uint32_t c = 0; c < f.channels; ++c) {
          const uint8_t* p = d + (uint64_t)i * f.block_align + (uint64_t)c * width;
          float v;
          if (flt && width == 4) {
            v = __builtin_bit_cast(float, le32(p));
          } else if (flt) {
            v = (float)__builtin_bit_cast(double, (uint64_t)le32(p) | ((uint64_t)le32(p + 4) << 32));
          } else if (width == 1) {
            v = (float)((int)p[0] - 128) / 128.f;
          } else if (width == 2) {
            v = (float)(int16_t)le16(p) / 32768.f;
          } else if (width == 3) {
            const int32_t s = (int32_t)(((uint32_t)p[0] << 8) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 24)) >> 8;
            v = (float)s / 8388608.f;
          } else {
            v = (float)(int32_t)le32(p) * (1.f / 2147483648.f);
          }
          acc = acc + v;
        }
        x[i] = acc / nch;
      }
      return TFP_OK;
    }
    pos = body + size + (size & 1);
  }
  return fail(TFP_E_FORMAT, have_fmt ? "no data chunk" : "no fmt chunk");
}

extern "C" int tfp_wav_read_f32(const char* path, float* x, int64_t cap, int64_t* nsamples, int32_t* sample_rate) {
  std::vector<uint8_t> buf;
  const int rc = read_file(path, buf);
  if (rc) return rc;
  return tfp_wav_decode_f32(buf.data(), (int64_t)buf.size(), x, cap, nsamples, sample_rate);
}

extern "C" int tfp_wav_read(const char* path, int16_t* pcm, int64_t cap, int64_t* nsamples, int32_t* sample_rate) {
  std::vector<uint8_t> buf;
  const int rc = read_file(path, buf);
  if (rc) return rc;
  return tfp_wav_decode(buf.data(), (int64_t)buf.size(), pcm, cap, nsamples, sample_rate);
}
