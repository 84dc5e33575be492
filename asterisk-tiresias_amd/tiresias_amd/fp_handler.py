"""Host-side mirror of the reference engine facade (/root/reference/src/fp_handler.h:13-38).

Same names, argument meaning and error behaviour as fp_handler.c, so tests read like the
reference's callers (application_handler.c, cli_handler.c, app_tiresias.c):
  * functions return True/False, a dict (the ast_json object) or None (NULL);
  * fp_search_fingerprint_info returns None for both "no match" and "error"
    (fp_handler.c:247-250, :386-390) and otherwise {uuid, name, context, hash,
    frame_count, match_count} (fp_handler.c:394-404);
  * fp_craete_audio_list_info (sic) returns True when the file is already enrolled
    (fp_handler.c:181-185).

The control plane (context_list / audio_list catalog, MD5 dedup, uuid v4) stays on SQLite,
as the reference keeps it; the hot path — fingerprinting and matching — runs on the GPU via
the C-ABI engine. fp_init/fp_term load and write the audio_recongition.db snapshot
(fp_handler.c:68-108) when a backup path is given — catalog tables to SQLite, fingerprint
rows straight into / out of the device index (dbio.py).
"""
from __future__ import annotations

import hashlib
import os
import sqlite3
import uuid as uuidlib
import wave

import numpy as np

from . import dbio
from ._lib import TfpError
from .engine import Engine, params, read_wav, read_wav_f32

TFP_E_FORMAT = -8

DEF_SEARCH_TOLERANCE = 0.001  # fp_handler.c:41
DEF_AUBIO_COEFS = 2           # fp_handler.c:39


def read_wav_mono16(filename: str):
    """aubio_source at the file's native rate (DEF_AUBIO_SAMPLERATE 0, fp_handler.c:37, :604):
    int16 PCM + rate, decoded by the engine library (tfp_wav_read). Raises TfpError for a
    missing file (TFP_E_NOENT) or audio the engine cannot take exactly (TFP_E_FORMAT)."""
    return read_wav(filename)


def read_audio(filename: str):
    """aubio_source's mono hop values of a WAV file: int16 PCM (tfp_wav_read) when they are int16
    steps (8/16-bit mono), else the fp32 values (tfp_wav_read_f32: multichannel mean, 24/32-bit,
    float). Raises TfpError (TFP_E_NOENT, TFP_E_FORMAT for non-WAV / unsupported encodings)."""
    try:
        return read_wav(filename)
    except TfpError as e:
        if e.code != TFP_E_FORMAT:
            raise
    return read_wav_f32(filename)


def write_wav_mono16(filename: str, pcm: np.ndarray, sample_rate: int = 8000):
    with wave.open(filename, "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(sample_rate)
        w.writeframes(np.ascontiguousarray(pcm, "<i2").tobytes())


class FpHandler:
    """One loaded module instance (g_db_ctx + the GPU engine)."""

    def __init__(self, device: int = 0, backup_path: str | None = None):
        """backup_path: the snapshot file (the reference hard-codes dbio.DEF_BACKUP_DATABASE);
        None keeps the state in memory only."""
        self.device = device
        self.backup_path = backup_path
        self.db = None
        self.engine = None

    # fp_handler.c:68-90 — init_database (the catalog tables) + engine, then the snapshot
    def fp_init(self) -> bool:
        self.db = sqlite3.connect(":memory:", check_same_thread=False)
        dbio.create_catalog(self.db)
        self.engine = Engine(self.device)
        if self.backup_path:
            try:
                dbio.load_backup(self.db, self.engine, self.backup_path)
            except Exception:
                return False  # "Could not load the database data."
        return True

    # fp_handler.c:92-108 — backup, then tear down
    def fp_term(self) -> bool:
        ok = True
        if self.backup_path and self.db and self.engine:
            try:
                dbio.write_backup(self.db, self.engine, self.backup_path)
            except Exception:
                ok = False  # "Could not write database."
        if self.engine:
            self.engine.close()
        self.engine = None
        if self.db:
            self.db.close()
        self.db = None
        return ok

    # ---- contexts (fp_handler.c:912-1095) ----------------------------------------------
    def fp_create_context_list_info(self, name: str, directory: str, replace: bool) -> bool:
        if name is None or directory is None:
            return False
        verb = "insert or replace" if replace else "insert"
        try:
            self.db.execute("%s into context_list(name, directory) values (?, ?);" % verb, (name, directory))
        except sqlite3.Error:
            return False
        return True

    def fp_delete_context_list_info(self, name: str) -> bool:
        if name is None:
            return False
        self.db.execute("delete from context_list where name = ?;", (name,))
        return True

    def fp_get_context_lists_all(self):
        return [dict(zip(("name", "directory"), r)) for r in self.db.execute("select * from context_list;")]

    def fp_get_context_list_info(self, name: str):
        r = self.db.execute("select * from context_list where name = ?;", (name,)).fetchone()
        return dict(zip(("name", "directory"), r)) if r else None

    # ---- audio list ---------------------------------------------------------------------
    def fp_get_audio_lists_all(self):
        return [self._audio_row(r) for r in self.db.execute("select * from audio_list;")]

    def fp_get_audio_lists_by_contextname(self, name: str):
        if name is None:
            return None
        return [self._audio_row(r) for r in self.db.execute("select * from audio_list where context = ?;", (name,))]

    @staticmethod
    def _audio_row(r):
        return dict(zip(("uuid", "name", "context", "hash"), r))

    def _audio_list_info(self, uuid: str):
        r = self.db.execute("select * from audio_list where uuid = ?;", (uuid,)).fetchone()
        return self._audio_row(r) if r else None

    @staticmethod
    def fp_generate_uuid() -> str:
        return str(uuidlib.uuid4())

    @staticmethod
    def fp_create_hash(filename: str):
        try:
            with open(filename, "rb") as f:
                return hashlib.md5(f.read()).hexdigest()
        except OSError:
            return None

    def fp_craete_audio_list_info(self, context: str, filename: str) -> bool:
        """fp_handler.c:161-197: catalog row (MD5 dedup per context) + fingerprint rows."""
        if context is None or filename is None:
            return False
        uuid = self.fp_generate_uuid()
        h = self.fp_create_hash(filename)
        if h is None:
            return False
        if self.db.execute("select * from audio_list where context = ? and hash = ?;", (context, h)).fetchone():
            return True  # already enrolled
        self.db.execute("insert into audio_list(uuid, name, context, hash) values (?, ?, ?, ?);",
                        (uuid, os.path.basename(filename), context, h))
        try:
            pcm, sr = read_audio(filename)
            fr = self._fingerprint(pcm, [0, len(pcm)], sr)
            self.engine.index_add(uuid, fr["m1"], fr["m2"])
        except Exception:
            self.fp_delete_audio_list_info(uuid)
            return False
        return True

    def _fingerprint(self, samples: np.ndarray, offsets, sr: int):
        if samples.dtype == np.float32:
            return self.engine.fingerprint_f32_batch(samples, offsets, sr)
        return self.engine.fingerprint_batch(samples, offsets, sr)

    def create_new_audio_info(self, context: str) -> bool:
        """app_tiresias.c:365-424 (the module's directory enrolment) batched onto the GPU.

        The reference scans the context's directory (alphasort, without "." and "..") and calls
        fp_craete_audio_list_info per file, skipping files that fail. Here the same catalog rows
        are written in the same order and with the same per-context MD5 dedup (also among the
        files of this scan). The fingerprints of all new files are computed by one
        tfp_fingerprint_batch call per sample rate and enrolled by one tfp_index_add_batch."""
        ctx = self.fp_get_context_list_info(context) if context is not None else None
        if ctx is None or ctx["directory"] is None:
            return False
        directory = ctx["directory"]
        try:
            names = sorted(n for n in os.listdir(directory) if n not in (".", ".."))
        except OSError:
            return False
        new = []  # (uuid, path, pcm, rate)
        seen = set()
        for name in names:
            path = "%s/%s" % (directory, name)
            h = self.fp_create_hash(path)
            if h is None:
                continue  # "Could not create fingerprint info."
            if h in seen or self.db.execute("select * from audio_list where context = ? and hash = ?;",
                                            (context, h)).fetchone():
                continue  # already enrolled
            try:
                pcm, sr = read_audio(path)
            except TfpError:
                continue
            uuid = self.fp_generate_uuid()
            self.db.execute("insert into audio_list(uuid, name, context, hash) values (?, ?, ?, ?);",
                            (uuid, os.path.basename(path), context, h))
            seen.add(h)
            new.append((uuid, pcm, sr))
        for sr, dt in sorted({(n[2], n[1].dtype.str) for n in new}):
            group = [n for n in new if n[2] == sr and n[1].dtype.str == dt]
            lens = [len(n[1]) for n in group]
            off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
            fr = self._fingerprint(np.concatenate([n[1] for n in group]), off, sr)
            foff = np.concatenate([[0], np.cumsum([(n + 255) // 256 for n in lens])]).astype(np.int64)
            self.engine.index_add_batch([n[0] for n in group], foff, fr["m1"], fr["m2"])
        return True

    def fp_delete_audio_list_info(self, uuid: str) -> bool:
        """fp_handler.c:115-159: audio_list row + its fingerprint rows."""
        if uuid is None:
            return False
        if self._audio_list_info(uuid) is None:
            return False
        self.db.execute("delete from audio_list where uuid = ?;", (uuid,))
        try:
            self.engine.index_remove(uuid)
        except Exception:
            pass  # no fingerprint rows (e.g. the fingerprint step failed)
        return True

    # ---- search (fp_handler.c:207-408) ------------------------------------------------
    def fp_search_fingerprint_info(self, context, filename, coefs, tolerance, freq_ignore_low, freq_ignore_high):
        if context is None or filename is None:
            return None
        if coefs < 1 or coefs > DEF_AUBIO_COEFS:
            return None
        try:
            pcm, sr = read_audio(filename)
        except TfpError:
            return None
        p = params(coefs, tolerance, freq_ignore_low, freq_ignore_high)
        if pcm.dtype == np.float32:
            res, _ = self.engine.search_f32_batch(pcm, [0, len(pcm)], p, sr)
        else:
            res, _ = self.engine.search_pcm_batch(pcm, [0, len(pcm)], p, sr)
        hit = res[0]
        if hit is None:
            return None
        info = self._audio_list_info(hit["audio_uuid"])
        if info is None:
            return None
        info["frame_count"] = hit["frame_count"]
        info["match_count"] = hit["match_count"]
        return info
