"""Hub resolution / downloader retries, tracing helpers (CPU)."""
import pytest

from llmss_amd.utils import hub
from llmss_amd.utils.tracing import PhaseTimer, range as trace_range


def test_weight_hub_files_filters():
    names = ["model-00001.safetensors", "training_args.safetensors", "model-00002.safetensors", "config.json"]
    got = hub.weight_hub_files("x/y", list_files=lambda mid, revision=None: names)
    assert got == ["model-00001.safetensors", "model-00002.safetensors"]
    got = hub.weight_hub_files("x/y", list_files=lambda mid, revision=None: ["pytorch_model.bin", "args.bin"])
    assert got == ["pytorch_model.bin"]
    with pytest.raises(FileNotFoundError):
        hub.weight_hub_files("x/y", list_files=lambda mid, revision=None: ["config.json"])


def test_download_retries_then_succeeds(tmp_path, monkeypatch):
    monkeypatch.setenv("HF_HUB_CACHE", str(tmp_path / "empty"))
    calls = {"n": 0}

    def fetch(repo_id, filename, revision=None):
        calls["n"] += 1
        if calls["n"] < 3:
            raise ConnectionError("flaky")
        p = tmp_path / filename
        p.write_bytes(b"x")
        return str(p)

    out = hub.download_weights(["a.safetensors"], "x/y", tries=5, backoff_s=0.0, fetch=fetch)
    assert calls["n"] == 3 and out[0].name == "a.safetensors"


def test_download_gives_up(tmp_path, monkeypatch):
    monkeypatch.setenv("HF_HUB_CACHE", str(tmp_path / "empty"))

    def fetch(**kw):
        raise ConnectionError("down")

    with pytest.raises(ConnectionError):
        hub.download_weights(["a.safetensors"], "x/y", tries=2, backoff_s=0.0, fetch=fetch)


def test_cache_hit_skips_fetch(tmp_path, monkeypatch):
    repo = tmp_path / "models--x--y"
    (repo / "snapshots" / "abc").mkdir(parents=True)
    (repo / "refs").mkdir()
    (repo / "refs" / "main").write_text("abc")
    (repo / "snapshots" / "abc" / "m.safetensors").write_bytes(b"x")
    monkeypatch.setenv("HF_HUB_CACHE", str(tmp_path))
    out = hub.download_weights(["m.safetensors"], "x/y", fetch=lambda **kw: pytest.fail("fetched"))
    assert out[0] == repo / "snapshots" / "abc" / "m.safetensors"


def test_offline_refuses(monkeypatch):
    monkeypatch.setenv("HF_HUB_OFFLINE", "1")
    with pytest.raises(FileNotFoundError):
        hub.weight_hub_files("x/y")


def test_phase_timer_cpu_noop():
    t = PhaseTimer(enabled=True)
    with t.phase("decode"):
        with trace_range("inner"):
            pass
    assert t.summary() == {}


def test_tokenizer_fallback_is_explicit(tmp_path):
    import pytest

    from llmss_amd.utils.tokenizer import ByteTokenizer, load_tokenizer

    assert isinstance(load_tokenizer("llama2-7b"), ByteTokenizer)  # preset name: synthetic model
    empty = tmp_path / "no_tok"
    empty.mkdir()
    assert isinstance(load_tokenizer(str(empty)), ByteTokenizer)  # checkpoint without tokenizer files
    broken = tmp_path / "broken"
    broken.mkdir()
    (broken / "tokenizer.json").write_text("{not json")
    with pytest.raises(RuntimeError):
        load_tokenizer(str(broken))


def test_stream_decoder_matches_full_decode():
    """Incremental detokenisation (gRPC GenerateStream): the streamed pieces concatenate to the full decode,
    with multi-byte characters split across tokens held back until complete."""
    import random

    from llmss_amd.utils.tokenizer import ByteTokenizer, StreamDecoder

    tok = ByteTokenizer()
    rnd = random.Random(0)
    alphabet = "ab é ö — ✓ 你好 🙂"
    for _ in range(20):
        text = "".join(rnd.choice(alphabet) for _ in range(rnd.randint(1, 40)))
        ids = tok.encode(text)
        d = StreamDecoder(tok)
        pieces = [d.push(i) for i in ids]
        assert "".join(pieces) + d.flush() == tok.decode(ids)
        assert all("�" not in p for p in pieces)
