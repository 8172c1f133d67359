"""`state.full(params, samples)` restated in numpy (oracle side).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restates whisper.cpp `whisper_full_with_state` as the reference drives it
(params from src/transcribe.rs:20-87: token_timestamps=true,
single_segment=true, suppress_blank=true, language option, DTW preset from
src/transcribe.rs:117-129).  SURVEY.md §3.2 / Appendix A.4-A.6:

  log-mel + signal energy -> [auto language detect: encode seek 0, decode [SOT]]
  -> seek loop over 30-s windows { encode; temperature loop { prefill
  [PREV, prompt_past[-n_take:], SOT, (lang, task)]; token loop: logit rules ->
  sample -> update seek_delta / completion }; rank; fallback check; emit
  segment; heuristic token timestamps; DTW re-forward + alignment }.

Implemented: greedy decoding at t = 0 with the fallback decision; sampling
at t > 0 and beam search are NOT in the oracle yet (tests run with the
fallback thresholds disabled, see `FullParams.synthetic_*`).

Synthetic workload pin, active when
`force_len > 0`: the window's decode is pinned to L tokens
[<|0.00|>, text x (L-3), <|t_end|>, EOT] — step 0 forces BEG, steps
1..L-3 mask EOT and timestamps, step L-2 forces the timestamp just below the
window end, step L-1 forces EOT.  The forcing is applied after whisper.cpp's
own logit rules, before the log-softmax.  L = round(3.3 * window_s) + 3.
"""
from __future__ import annotations

import dataclasses
import math

import numpy as np

from . import dtw as dtwmod
from .mel import log_mel, mel_lengths, signal_energy
from .model import DecoderState, Whisper
from .vocab import LANGS, Vocab

CHUNK = 30
N_FRAMES = 3000            # 100 * WHISPER_CHUNK_SIZE
DELTA_MIN = 10

ALIGNMENT_HEADS = {        # whisper.cpp g_aheads_* (from OpenAI _ALIGNMENT_HEADS); unverified offline
    "tiny.en": [(1, 0), (2, 0), (2, 5), (3, 0), (3, 1), (3, 2), (3, 3), (3, 4)],
    "tiny": [(2, 2), (3, 0), (3, 2), (3, 3), (3, 4), (3, 5)],
    "base.en": [(3, 3), (4, 7), (5, 1), (5, 5), (5, 7)],
    "base": [(3, 1), (4, 2), (4, 3), (4, 7), (5, 1), (5, 2), (5, 4), (5, 6)],
    "small.en": [(6, 6), (7, 0), (7, 3), (7, 8), (8, 2), (8, 5), (8, 7), (9, 0), (9, 4), (9, 8), (9, 10),
                 (10, 0), (10, 1), (10, 2), (10, 3), (10, 6), (10, 11), (11, 2), (11, 4)],
    "small": [(5, 3), (5, 9), (8, 0), (8, 4), (8, 7), (8, 8), (9, 0), (9, 7), (9, 9), (10, 5)],
    "medium.en": [(11, 4), (14, 1), (14, 12), (14, 14), (15, 4), (16, 0), (16, 4), (16, 9), (17, 12),
                  (17, 14), (18, 7), (18, 10), (18, 15), (20, 0), (20, 3), (20, 9), (20, 14), (21, 12)],
    "medium": [(13, 15), (15, 4), (15, 15), (16, 1), (20, 0), (23, 4)],
    "large-v3": [(7, 0), (10, 17), (12, 18), (13, 12), (16, 1), (17, 14), (19, 11), (21, 4), (24, 1), (25, 6)],
    "large-v3-turbo": [(2, 4), (2, 11), (3, 3), (3, 6), (3, 11), (3, 14)],
    # reduced test configs: every head of the upper half of the decoder (whisper.cpp N_TOP_MOST style)
    "tiny-test": [(1, 0), (1, 1)],
    "tiny-test-ml": [(1, 0), (1, 1)],
}


def aheads_for_model_name(name: str):
    """src/transcribe.rs:117-129: unknown names fall back to the Small preset."""
    return ALIGNMENT_HEADS.get(name, ALIGNMENT_HEADS["small"])


@dataclasses.dataclass
class FullParams:
    strategy: str = "beam"           # src/transcribe.rs:25-33 ("greedy" only if requested)
    best_of: int = 5
    beam_size: int = 5
    language: str = "auto"
    translate: bool = False
    n_max_text_ctx: int = 16384
    initial_prompt: str | None = None
    temperature: float = 0.0
    temperature_inc: float = 0.2
    entropy_thold: float = 2.4
    logprob_thold: float = -1.0
    no_speech_thold: float = 0.6
    thold_pt: float = 0.01
    thold_ptsum: float = 0.01
    max_initial_ts: float = 1.0
    length_penalty: float = -1.0
    suppress_blank: bool = True
    single_segment: bool = True
    token_timestamps: bool = True
    max_tokens: int = 0
    force_len_rate: float = 0.0      # synthetic pin: L = round(rate * window_s) + 3 (0 = off)


@dataclasses.dataclass
class Token:
    id: int
    tid: int = 0
    p: float = 0.0
    plog: float = 0.0
    pt: float = 0.0
    ptsum: float = 0.0
    t0: int = -1
    t1: int = -1
    t_dtw: int = -1
    vlen: float = 0.0
    margin: float = float("inf")   # test diagnostics: logprob gap top-1 - top-2 at the greedy pick


@dataclasses.dataclass
class Result:
    t0: int
    t1: int
    text: str
    tokens: list


def voice_length(text: str) -> float:
    res = np.float32(0.0)
    for c in text:
        if c == ' ':
            add = 0.01
        elif c == ',':
            add = 2.0
        elif c in '.!?':
            add = 3.0
        elif '0' <= c <= '9':
            add = 3.0
        else:
            add = 1.0
        res = np.float32(res + np.float32(add))
    return float(res)


def c_round(x: float) -> int:
    return int(math.floor(x + 0.5)) if x >= 0 else -int(math.floor(-x + 0.5))


class WhisperState:
    """whisper_state: persists across `full` calls of one run (src/transcribe.rs:335)."""

    def __init__(self, model: Whisper, vocab: Vocab, model_name: str, dtw: bool = True):
        self.m, self.v = model, vocab
        self.aheads = aheads_for_model_name(model_name) if dtw else None
        self.t_beg = 0
        self.t_last = 0
        self.tid_last = 0
        self.lang_id = 0
        self.result_all = []
        self.stats = {"encode": 0, "decode_tokens": 0, "decode_calls": 0, "no_speech_skips": 0, "fallbacks": 0}
        self.lang_margin = float("inf")   # test diagnostics: language logit gap top-1 - top-2
        # whisper_decoder::rng (std::mt19937): decoder 0 seeded once per state, decoders >= 1
        # re-seeded with 0 on every whisper_full call (WHISPER_DECODER_INIT) -- parity unpinned
        self.rngs = [np.random.RandomState(0)] + [None] * 15

    # ------------------------------------------------------------ logits
    def process_logits(self, logits, tokens_cur, has_ts, seek_delta, params, temperature, force):
        v = self.v
        logits = logits.astype(np.float32).copy()
        n = logits.shape[0]
        if temperature > 0:
            logits /= np.float32(temperature)
        is_initial = len(tokens_cur) == 0
        if params.suppress_blank and is_initial:
            logits[v.eot] = -np.inf
            logits[v.token_to_id[" "]] = -np.inf
        logits[v.not_] = -np.inf
        logits[v.sot] = -np.inf
        logits[v.nosp] = -np.inf
        logits[v.solm] = -np.inf
        logits[v.translate] = -np.inf
        logits[v.transcribe] = -np.inf
        logits[v.prev] = -np.inf
        for i in range(len(LANGS)):
            logits[v.token_lang(i)] = -np.inf
        last_ts = len(tokens_cur) > 0 and tokens_cur[-1].id >= v.beg
        pen_ts = len(tokens_cur) < 2 or tokens_cur[-2].id >= v.beg
        if last_ts:
            if pen_ts:
                logits[v.beg:] = -np.inf
            else:
                logits[:v.eot] = -np.inf
        if is_initial and params.max_initial_ts > 0:
            precision = np.float32(CHUNK) / np.float32(self.m.hp.n_audio_ctx)
            tid0 = c_round(float(np.float32(params.max_initial_ts) / precision))
            logits[v.beg + tid0 + 1:] = -np.inf
        if has_ts:
            tid0 = seek_delta // 2
            logits[v.beg:v.beg + tid0] = -np.inf
        if force is not None:
            kind, val = force
            if kind == "only":
                keep = logits[val]
                logits[:] = -np.inf
                logits[val] = 0.0 if not np.isfinite(keep) else keep
            elif kind == "text":
                logits[v.eot] = -np.inf
                logits[v.beg:] = -np.inf
        logprobs = compute_logprobs(logits)
        # timestamp_logprob > max text logprob -> mask text
        lp_ts = logprobs[v.beg:]
        lmax = lp_ts.max()
        fin = lp_ts[lp_ts > -np.inf]
        s = np.float32(np.exp(fin - lmax).astype(np.float32).sum(dtype=np.float32)) if fin.size else np.float32(0)
        ts_lp = np.float32(np.log(s) + lmax) if s > 0 else -np.inf
        max_text = logprobs[:v.beg].max()
        if ts_lp > max_text:
            logits[:v.beg] = -np.inf
            logprobs[:v.beg] = -np.inf
        probs = np.where(logits == -np.inf, np.float32(0), np.exp(logprobs)).astype(np.float32)
        return logits, logprobs, probs

    def sample_greedy(self, probs, logprobs):
        v = self.v
        ts = probs[v.beg:].astype(np.float64)
        sum_ts = float(ts.sum())
        tid = 0
        max_ts = 0.0
        if ts.size and ts.max() > 0:
            tid = v.beg + int(np.argmax(ts))
            max_ts = float(ts.max())
        tok = Token(id=0, tid=tid, pt=float(max_ts / (sum_ts + 1e-10)), ptsum=sum_ts)
        idx = int(np.argmax(probs))
        if probs[idx] > 0:
            tok.id, tok.p, tok.plog = idx, float(probs[idx]), float(logprobs[idx])
            fin = logprobs[logprobs > -np.inf]
            if fin.size > 1:
                top2 = np.partition(fin, -2)[-2:]
                tok.margin = float(top2[1] - top2[0])
        if tok.id >= v.beg:
            tok.tid = tok.id
            tok.pt = tok.p
        return tok

    # ------------------------------------------------------------ full
    def full(self, samples: np.ndarray, params: FullParams):
        v, m, hp = self.v, self.m, self.m.hp
        self.result_all = []
        for j in range(1, len(self.rngs)):
            self.rngs[j] = np.random.RandomState(0)
        n = samples.shape[0]
        mel = log_mel(samples, hp.n_mels)
        energy = None
        if params.token_timestamps:
            self.t_beg = self.t_last = self.tid_last = 0
            if n > 0:
                energy = signal_energy(samples)
        _, n_len_org = mel_lengths(n)
        seek_start, seek_end = 0, n_len_org
        if seek_end < seek_start + DELTA_MIN:
            return 0

        prompt_past = []                         # no_context = true
        if params.initial_prompt:
            prompt_past = v.tokenize(params.initial_prompt) + prompt_past

        enc_cache = {}

        def encode(seek):
            if seek not in enc_cache:
                win = mel[:, seek:seek + N_FRAMES]
                if win.shape[1] < N_FRAMES:
                    win = np.concatenate([win, np.zeros((win.shape[0], N_FRAMES - win.shape[1]), np.float32)], 1)
                enc = m.encode(win)
                enc_cache.clear()
                enc_cache[seek] = m.cross_kv(enc)
                self.stats["encode"] += 1
            return enc_cache[seek]

        language = params.language
        if language in (None, "", "auto"):
            cross = encode(seek_start)
            st = DecoderState(m)
            logits = st.forward([v.sot], cross)
            self.stats["decode_calls"] += 1
            lang_logits = [(float(logits[v.token_lang(i)]), i) for i in range(len(LANGS))]
            best = max(lang_logits, key=lambda t: t[0])     # sort descending, take first
            self.lang_id = best[1]
            ll = sorted((x for x, _ in lang_logits), reverse=True)
            self.lang_margin = ll[0] - ll[1]
            language = LANGS[self.lang_id]
        prompt_init = [v.sot]
        if v.multilingual:
            self.lang_id = LANGS.index(language)
            prompt_init.append(v.token_lang(self.lang_id))
            prompt_init.append(v.translate if params.translate else v.transcribe)

        temps = []
        if params.temperature_inc > 0:
            t = params.temperature
            while t < 1.0 + 1e-6:
                temps.append(t)
                t = float(np.float32(t) + np.float32(params.temperature_inc))
        else:
            temps = [params.temperature]

        seek = seek_start
        n_text_ctx = hp.n_text_ctx
        while True:
            if seek + 100 >= seek_end:
                break
            cross = encode(seek)
            if seek > seek_start and seek + 500 >= seek_end:
                prompt_past = []
            best = None
            for it, t_cur in enumerate(temps):
                prompt = []
                if prompt_past and t_cur < 0.5 and params.n_max_text_ctx > 0:
                    n_take = min(min(params.n_max_text_ctx, n_text_ctx // 2), len(prompt_past))
                    prompt = [v.prev] + prompt_past[len(prompt_past) - n_take:]
                prompt = prompt + prompt_init
                st = DecoderState(m)
                logits = st.forward(prompt, cross)
                self.stats["decode_calls"] += 1
                self.stats["decode_tokens"] += len(prompt)
                lp = compute_logprobs(logits.astype(np.float32))
                no_speech_prob = float(np.exp(lp[v.nosp]))
                window = min(seek_end - seek, N_FRAMES)
                L = 0
                if params.force_len_rate > 0:
                    L = max(3, c_round(params.force_len_rate * window / 100.0) + 3)
                seq = dict(tokens=[], result_len=0, seek_delta=N_FRAMES, has_ts=False,
                           failed=False, completed=False)
                n_max = n_text_ctx // 2 - 4
                single = params.strategy == "greedy" and t_cur <= 0
                if t_cur > 0:
                    seq = self.decode_sample(st, logits, cross, params, t_cur, seek, seek_end, L, window)
                elif params.strategy != "greedy":
                    seq = self.decode_beam(st, logits, cross, prompt, params, t_cur, seek, seek_end, L, window)
                for i in range(n_max if single else 0):
                    force = None
                    if L:
                        if i == 0:
                            force = ("only", v.beg)
                        elif i < L - 2:
                            force = ("text", None)
                        elif i == L - 2:
                            force = ("only", v.beg + min(1500, max(1, (window - DELTA_MIN - 1) // 2)))
                        else:
                            force = ("only", v.eot)
                    _, lps, probs = self.process_logits(logits, seq["tokens"], seq["has_ts"], seq["seek_delta"],
                                                        params, t_cur, force)
                    tok = self.sample_greedy(probs, lps)
                    seq["tokens"].append(tok)
                    # update decoder state
                    if tok.id > v.beg:
                        sdn = 2 * (tok.id - v.beg)
                        if seq["has_ts"] and seq["seek_delta"] > sdn and seq["result_len"] < i:
                            seq["failed"] = True
                            break
                        seq["seek_delta"] = sdn
                        seq["result_len"] = i + 1
                        seq["has_ts"] = True
                    if (tok.id == v.eot or (params.max_tokens > 0 and i >= params.max_tokens)
                            or (seq["has_ts"] and seek + seq["seek_delta"] + DELTA_MIN >= seek_end)):
                        if seq["result_len"] == 0:
                            if seek + seq["seek_delta"] + DELTA_MIN >= seek_end:
                                seq["result_len"] = i + 1
                            else:
                                seq["failed"] = True
                                break
                        if params.single_segment:
                            seq["result_len"] = i + 1
                            seq["seek_delta"] = N_FRAMES
                        seq["completed"] = True
                        break
                    if i == n_max - 1 and (seq["result_len"] == 0 or seq["seek_delta"] < N_FRAMES // 2):
                        seq["failed"] = True
                        break
                    logits = st.forward([tok.id], cross)
                    self.stats["decode_calls"] += 1
                    self.stats["decode_tokens"] += 1
                # rank (single decoder)
                if single:
                    seq["tokens"] = seq["tokens"][:seq["result_len"]]
                    score_sequence(seq, params)
                    if seq["failed"] is False and seq["result_len"] > 32 and seq["entropy"] < params.entropy_thold:
                        seq["failed"] = True
                seq["no_speech_prob"] = no_speech_prob
                best = seq
                success = True
                if it != len(temps) - 1:
                    if seq["failed"] or (seq["avg_logprobs"] < params.logprob_thold
                                         and no_speech_prob < params.no_speech_thold):
                        success = False
                if success:
                    break
                self.stats["fallbacks"] += 1
            # ---------------- output
            seek_delta = best["seek_delta"]
            result_len = best["result_len"]
            tokens_cur = best["tokens"]
            n_before = len(self.result_all)
            is_no_speech = (best["no_speech_prob"] > params.no_speech_thold
                            and best["avg_logprobs"] < params.logprob_thold)
            new_past = []
            if prompt and prompt[0] == v.prev:
                new_past = prompt[1:len(prompt) - len(prompt_init)]
            if not is_no_speech:
                new_past += [t.id for t in tokens_cur[:result_len]]
            else:
                self.stats["no_speech_skips"] += 1
            prompt_past = new_past
            if tokens_cur and not is_no_speech:
                t0 = seek + 2 * (tokens_cur[0].tid - v.beg)
                text = "".join(v.id_to_token[t.id] for t in tokens_cur if t.id < v.eot)
                if text:
                    t1 = seek + seek_delta
                    self.result_all.append(Result(t0, t1, text, [dataclasses.replace(t) for t in tokens_cur]))
                    if params.token_timestamps:
                        self.token_timestamps_heuristic(len(self.result_all) - 1, params, energy)
            n_new = len(self.result_all) - n_before
            if self.aheads and n_new:
                n_frames = min(min(N_FRAMES, seek_delta), seek_end - seek)
                self.dtw_timestamps(n_before, n_new, seek, n_frames, cross, language)
            if (len(tokens_cur) > 1 and tokens_cur[-2].id < v.beg and tokens_cur[-1].id > v.beg):
                seek_delta = min(seek_end - seek, N_FRAMES)
            seek += seek_delta
        return 0

    # ------------------------------------------------------------ temperature sampling
    @staticmethod
    def discrete_draw(rs, weights):
        """libstdc++ std::discrete_distribution<int>(w.begin(), w.end())(mt19937): sequential
        double sum, normalise, sequential partial sums with the last set to 1, then
        lower_bound of generate_canonical<double, 53> (two 32-bit draws)."""
        w = np.asarray(weights, np.float32).astype(np.float64)
        tot = np.cumsum(w)[-1]
        cp = np.cumsum(w / tot)
        cp[-1] = 1.0
        x0, x1 = rs.randint(0, 2 ** 32, size=2, dtype=np.uint32)
        u = (float(x0) + float(x1) * 4294967296.0) / 18446744073709551616.0
        if u >= 1.0:
            u = np.nextafter(1.0, 0.0)
        return int(np.searchsorted(cp, u, side="left"))

    def decode_sample(self, st, logits, cross, params, t_cur, seek, seek_end, L, window):
        """t > 0: best_of decoders share the prompt; each draws with its own rng
        (whisper_sample_token, best = false); ranking as decode_beam."""
        v = self.v
        K = max(1, params.best_of)
        n_max = self.m.hp.n_text_ctx // 2 - 4
        dec = [dict(tokens=[], result_len=0, seek_delta=N_FRAMES, has_ts=False, failed=False, completed=False)
               for _ in range(K)]
        states = [st] + [st.copy() for _ in range(K - 1)]
        row_logits = [logits] * K
        for i in range(n_max):
            act = [j for j in range(K) if not dec[j]["completed"] and not dec[j]["failed"]]
            if not act:
                break
            force = None
            if L:
                if i == 0:
                    force = ("only", v.beg)
                elif i < L - 2:
                    force = ("text", None)
                elif i == L - 2:
                    force = ("only", v.beg + min(1500, max(1, (window - DELTA_MIN - 1) // 2)))
                else:
                    force = ("only", v.eot)
            for j in act:
                d = dec[j]
                _, lps, probs = self.process_logits(row_logits[j], d["tokens"], d["has_ts"], d["seek_delta"],
                                                    params, t_cur, force)
                ts = probs[v.beg:].astype(np.float64)
                sum_ts = float(np.cumsum(ts)[-1]) if ts.size else 0.0
                mx = float(ts.max()) if ts.size else 0.0
                tid = v.beg + int(np.argmax(ts)) if mx > 0 else 0
                tok = Token(id=self.discrete_draw(self.rngs[j], probs), tid=tid, pt=float(mx / (sum_ts + 1e-10)),
                            ptsum=sum_ts)
                tok.p, tok.plog = float(probs[tok.id]), float(lps[tok.id])
                if tok.id >= v.beg:
                    tok.tid, tok.pt = tok.id, tok.p
                d["tokens"].append(tok)
            for j in act:
                d = dec[j]
                tok = d["tokens"][-1]
                if tok.id > v.beg:
                    sdn = 2 * (tok.id - v.beg)
                    if d["has_ts"] and d["seek_delta"] > sdn and d["result_len"] < i:
                        d["failed"] = True
                        continue
                    d["seek_delta"] = sdn
                    d["result_len"] = i + 1
                    d["has_ts"] = True
                if (tok.id == v.eot or (params.max_tokens > 0 and i >= params.max_tokens)
                        or (d["has_ts"] and seek + d["seek_delta"] + DELTA_MIN >= seek_end)):
                    if d["result_len"] == 0:
                        if seek + d["seek_delta"] + DELTA_MIN >= seek_end:
                            d["result_len"] = i + 1
                        else:
                            d["failed"] = True
                            continue
                    if params.single_segment:
                        d["result_len"] = i + 1
                        d["seek_delta"] = N_FRAMES
                    d["completed"] = True
                    continue
                if i == n_max - 1 and (d["result_len"] == 0 or d["seek_delta"] < N_FRAMES // 2):
                    d["failed"] = True
            for j in [j for j in act if not dec[j]["completed"] and not dec[j]["failed"]]:
                row_logits[j] = states[j].forward([dec[j]["tokens"][-1].id], cross)
                self.stats["decode_calls"] += 1
                self.stats["decode_tokens"] += 1
        best, best_score = 0, -np.inf
        for j, d in enumerate(dec):
            if d["failed"]:
                continue
            d["tokens"] = d["tokens"][:d["result_len"]]
            score_sequence(d, params)
            if d["result_len"] > 32 and d["entropy"] < params.entropy_thold:
                d["failed"] = True
                continue
            if best_score < d["score"]:
                best, best_score = j, d["score"]
        out = dec[best]
        out["tokens"] = out["tokens"][:out["result_len"]]
        score_sequence(out, params)
        return out

    # ------------------------------------------------------------ beam search
    def topk(self, logprobs, k):
        """whisper_sample_token_topk over the processed logits: descending, ties by lower
        token id; only finite entries are candidates (with the synthetic forcing a row can
        have fewer than k; whisper.cpp would pad with -inf entries that are never chosen
        while a finite candidate exists)."""
        fin = np.nonzero(logprobs > -np.inf)[0]
        order = fin[np.lexsort((fin, -logprobs[fin].astype(np.float64)))]
        return [int(i) for i in order[:k]]

    def decode_beam(self, st, logits, cross, prompt, params, t_cur, seek, seek_end, L, window):
        """whisper.cpp WHISPER_SAMPLING_BEAM_SEARCH at t = 0 (patience -1): K decoders share
        the prompt; each live decoder proposes its top-K tokens; candidates are ordered by
        cumulative log-probability (stable: decoder index, then rank), duplicate sequences are
        dropped, and live decoders take the candidates in order,
        wrapping around when there are fewer; KV caches follow their parents.  Ranking:
        score = sum logprob / length (length_penalty -1), entropy check, first best wins."""
        v = self.v
        K = max(1, params.beam_size)
        n_max = self.m.hp.n_text_ctx // 2 - 4
        dec = [dict(tokens=[], result_len=0, seek_delta=N_FRAMES, has_ts=False, failed=False, completed=False,
                    sum_all=0.0) for _ in range(K)]
        states = [st] + [st.copy() for _ in range(K - 1)]
        row_logits = [logits] * K
        self._no_speech = None
        for i in range(n_max):
            act = [j for j in range(K) if not dec[j]["completed"] and not dec[j]["failed"]]
            if not act:
                break
            force = None
            if L:
                if i == 0:
                    force = ("only", v.beg)
                elif i < L - 2:
                    force = ("text", None)
                elif i == L - 2:
                    force = ("only", v.beg + min(1500, max(1, (window - DELTA_MIN - 1) // 2)))
                else:
                    force = ("only", v.eot)
            cands = []
            for j in act:
                d = dec[j]
                _, lps, probs = self.process_logits(row_logits[j], d["tokens"], d["has_ts"], d["seek_delta"],
                                                    params, t_cur, force)
                g = self.sample_greedy(probs, lps)
                for tid in self.topk(lps, K):
                    tok = Token(id=tid, tid=g.tid, p=float(probs[tid]), plog=float(lps[tid]), pt=g.pt, ptsum=g.ptsum)
                    if tok.id >= v.beg:
                        tok.tid, tok.pt = tok.id, tok.p
                    cands.append((j, d["sum_all"] + tok.plog, tok))
            cands.sort(key=lambda c: -c[1])          # stable
            uniq = []
            for c in cands:
                key = [t.id for t in dec[c[0]]["tokens"]] + [c[2].id]
                if all(key != [t.id for t in dec[u[0]]["tokens"]] + [u[2].id] for u in uniq):
                    uniq.append(c)
            nd, ns = list(dec), list(states)
            cur = 0
            for j in act:
                if cur >= len(uniq):
                    cur = 0
                pj, sm, tok = uniq[cur]
                cur += 1
                nd[j] = dict(dec[pj], tokens=list(dec[pj]["tokens"]) + [tok], sum_all=sm)
                ns[j] = states[pj].copy() if pj != j else states[j]
            dec, states = nd, ns
            for j in act:
                d = dec[j]
                tok = d["tokens"][-1]
                if tok.id > v.beg:
                    sdn = 2 * (tok.id - v.beg)
                    if d["has_ts"] and d["seek_delta"] > sdn and d["result_len"] < i:
                        d["failed"] = True
                        continue
                    d["seek_delta"] = sdn
                    d["result_len"] = i + 1
                    d["has_ts"] = True
                if (tok.id == v.eot or (params.max_tokens > 0 and i >= params.max_tokens)
                        or (d["has_ts"] and seek + d["seek_delta"] + DELTA_MIN >= seek_end)):
                    if d["result_len"] == 0:
                        if seek + d["seek_delta"] + DELTA_MIN >= seek_end:
                            d["result_len"] = i + 1
                        else:
                            d["failed"] = True
                            continue
                    if params.single_segment:
                        d["result_len"] = i + 1
                        d["seek_delta"] = N_FRAMES
                    d["completed"] = True
                    continue
                if i == n_max - 1 and (d["result_len"] == 0 or d["seek_delta"] < N_FRAMES // 2):
                    d["failed"] = True
            live = [j for j in act if not dec[j]["completed"] and not dec[j]["failed"]]
            for j in live:
                row_logits[j] = states[j].forward([dec[j]["tokens"][-1].id], cross)
                self.stats["decode_calls"] += 1
                self.stats["decode_tokens"] += 1
        best, best_score = 0, -np.inf
        for j, d in enumerate(dec):
            if d["failed"]:
                continue
            d["tokens"] = d["tokens"][:d["result_len"]]
            score_sequence(d, params)
            if d["result_len"] > 32 and d["entropy"] < params.entropy_thold:
                d["failed"] = True
                continue
            if best_score < d["score"]:
                best, best_score = j, d["score"]
        out = dec[best]
        out["tokens"] = out["tokens"][:out["result_len"]]
        score_sequence(out, params)
        return out

    # ------------------------------------------------------------ timestamps
    def token_timestamps_heuristic(self, i_segment, params, energy):
        v = self.v
        seg = self.result_all[i_segment]
        toks = seg.tokens
        n_samples = energy.shape[0]
        t0, t1 = seg.t0, seg.t1
        n = len(toks)
        if n == 0:
            return
        if n == 1:
            toks[0].t0, toks[0].t1 = t0, t1
            return
        for j in range(n):
            tk = toks[j]
            if j == 0:
                if tk.id == v.beg:
                    toks[0].t0 = t0
                    toks[0].t1 = t0
                    toks[1].t0 = t0
                    self.t_beg = t0
                    self.t_last = t0
                    self.tid_last = v.beg
                else:
                    toks[0].t0 = self.t_last
            tt = self.t_beg + 2 * (tk.tid - v.beg)
            tk.vlen = voice_length(v.id_to_token[tk.id])
            if (np.float32(tk.pt) > np.float32(params.thold_pt) and np.float32(tk.ptsum) > np.float32(params.thold_ptsum)
                    and tk.tid > self.tid_last and tt <= t1):
                if j > 0:
                    toks[j - 1].t1 = tt
                tk.t0 = tt
                self.tid_last = tk.tid
        toks[n - 2].t1 = t1
        toks[n - 1].t0 = t1
        toks[n - 1].t1 = t1
        self.t_last = t1
        p0 = p1 = 0
        while True:
            while p1 < n and toks[p1].t1 < 0:
                p1 += 1
            if p1 >= n:
                p1 -= 1
            if p1 > p0:
                psum = 0.0
                for j in range(p0, p1 + 1):
                    psum += toks[j].vlen
                dt = float(toks[p1].t1 - toks[p0].t0)
                for j in range(p0 + 1, p1 + 1):
                    ct = toks[j - 1].t0 + dt * toks[j - 1].vlen / psum
                    toks[j - 1].t1 = int(ct)
                    toks[j].t0 = int(ct)
            p1 += 1
            p0 = p1
            if p1 >= n:
                break
        for j in range(n - 1):
            if toks[j].t1 < 0:
                toks[j + 1].t0 = toks[j].t1
            if j > 0:
                if toks[j - 1].t1 > toks[j].t0:
                    toks[j].t0 = toks[j - 1].t1
                    toks[j].t1 = max(toks[j].t0, toks[j].t1)
        hw = 16000 // 8

        def ts2s(t):
            return max(0, min(n_samples - 1, (t * 16000) // 100))

        def s2ts(i):
            return (100 * i) // 16000
        for j in range(n):
            if toks[j].id >= v.eot:
                continue
            s0 = ts2s(toks[j].t0)
            s1 = ts2s(toks[j].t1)
            ss0 = max(s0 - hw, 0)
            ss1 = min(s1 + hw, n_samples)
            ns = ss1 - ss0
            ssum = np.float32(0)
            for k in range(ss0, ss1):
                ssum = np.float32(ssum + energy[k])
            thold = np.float32(0.5 * float(ssum) / ns)
            k = s0
            if energy[k] > thold and j > 0:
                while k > 0 and energy[k] > thold:
                    k -= 1
                toks[j].t0 = s2ts(k)
                if toks[j].t0 < toks[j - 1].t1:
                    toks[j].t0 = toks[j - 1].t1
                else:
                    s0 = k
            else:
                while energy[k] < thold and k < s1:
                    k += 1
                s0 = k
                toks[j].t0 = s2ts(k)
            k = s1
            if energy[k] > thold:
                while k < n_samples - 1 and energy[k] > thold:
                    k += 1
                toks[j].t1 = s2ts(k)
                if j < ns - 1 and j + 1 < n and toks[j].t1 > toks[j + 1].t0:
                    toks[j].t1 = toks[j + 1].t0
                else:
                    s1 = k
            else:
                while energy[k] < thold and k > s0:
                    k -= 1
                s1 = k
                toks[j].t1 = s2ts(k)

    def dtw_timestamps(self, i_segment, n_segments, seek, n_frames, cross, language):
        v = self.v
        tokens = [v.sot]
        if v.multilingual:
            tokens.append(v.token_lang(LANGS.index(language)))
        sot_len = len(tokens)
        tokens.append(v.not_)
        for s in self.result_all[i_segment:i_segment + n_segments]:
            tokens += [t.id for t in s.tokens if t.id < v.eot]
        tokens.append(v.eot)
        st = DecoderState(self.m)
        _, qk = st.forward(tokens, cross, want_logits=None, aheads=self.aheads)
        self.stats["decode_calls"] += 1
        self.stats["decode_tokens"] += len(tokens)
        x = dtwmod.alignment_matrix(qk, n_frames, sot_len)
        times = dtwmod.token_times(x, seek)
        it = iter([t for s in self.result_all[i_segment:i_segment + n_segments] for t in s.tokens if t.id < v.eot])
        for ts in times:
            tok = next(it)
            tok.t_dtw = ts


def compute_logprobs(logits):
    logits = logits.astype(np.float32)
    lmax = logits.max()
    fin = logits > -np.inf
    s = np.exp(logits[fin] - lmax).astype(np.float32).sum(dtype=np.float32)
    lse = np.float32(np.log(s) + lmax)
    out = np.full_like(logits, -np.inf)
    out[fin] = logits[fin] - lse
    return out


def score_sequence(seq, params):
    rl = seq["result_len"]
    seq.setdefault("avg_logprobs", -np.inf)
    seq.setdefault("entropy", 0.0)
    seq.setdefault("score", -np.inf)
    if rl == 0:
        return
    res = 0.0
    for t in seq["tokens"][:rl]:
        res += t.plog
    seq["sum_logprobs"] = res
    seq["avg_logprobs"] = res / rl
    pen = rl
    if params.length_penalty > 0:
        pen = ((5.0 + pen) / 6.0) ** params.length_penalty
    seq["score"] = res / pen
    cnt = {}
    for t in seq["tokens"][max(0, rl - 32):rl]:
        cnt[t.id] = cnt.get(t.id, 0) + 1
    tot = sum(cnt.values())
    ent = 0.0
    for k in sorted(cnt):
        p = cnt[k] / tot
        ent -= p * math.log(p)
    seq["entropy"] = ent
