"""CPU oracle for the whisper-diarize-rs hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product path (libwdr.so, the `wdr`
Python mirror) imports, links or executes anything in this package.  Only
`tests/`, `__graft_entry__.smoke()` and the `cpu_baseline` leg of `bench.py`
may use it, and there only as the checker / the timed CPU restatement.

What it restates (every function cites the reference
call site it stands for):

* the reference crate's own Rust glue (src/vad.rs:33-84,
  src/transcribe.rs:171-320,376-523, src/engine.rs:89-147) — restated
  exactly;
* whisper.cpp / ggml behaviour invoked through whisper-rs 0.15.0
  (whisper-rs-sys 0.14.0 @ 0c509ec9): log-mel, encoder/decoder numerics,
  logit rules, greedy decode loop, heuristic token timestamps, DTW — restated
  from the published algorithm; whisper.cpp sources are NOT present in this
  container, so that part is *parity unpinned* against whisper.cpp itself and
  pinned only against third-party golden vectors (transformers 5.15.0: mel
  filters, DTW recurrence, median filter, Whisper layer math) committed under
  tests/golden/.
"""
