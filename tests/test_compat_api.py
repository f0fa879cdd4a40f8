"""Reference API compatibility: MODEL_REGISTRY façade (HF-style forward with past_key_values) and the
generate.py CLI (same flags, same three stdout lines), on CPU at TP=1 (BASELINE config #1 plumbing)."""
import subprocess
import sys

import torch
from transformers import AutoConfig

from helpers import save_hf_model


def test_model_registry_facade(tmp_path):
    from llmss.server.models.custom_modeling import MODEL_REGISTRY
    from llmss.server.models.utils.hub import weight_files
    from llmss.server.models.utils.weights import Weights

    for name in ("gptj", "gpt2", "llama"):
        d = str(tmp_path / name)
        hf = save_hf_model(name, d)
        config = AutoConfig.from_pretrained(d)
        w = Weights(weight_files(d), torch.device("cpu"), torch.float32, None)
        model = MODEL_REGISTRY[config.model_type](config, w)
        model.eval()
        ids = torch.randint(0, 100, (2, 7))
        out = model(ids, past_key_values=None, use_cache=True)
        with torch.no_grad():
            ref = hf(ids).logits
        assert out.logits.shape == ref.shape
        assert (out.logits - ref).abs().max() < 1e-4
        nxt = ref[:, -1].argmax(-1, keepdim=True)
        out2 = model(nxt, past_key_values=out.past_key_values, use_cache=True)
        with torch.no_grad():
            ref2 = hf(torch.cat([ids, nxt], 1)).logits[:, -1:]
        assert (out2.logits - ref2).abs().max() < 1e-4
        out3 = model(ids, labels=ids)
        assert out3.loss is not None and torch.isfinite(out3.loss)


def test_generate_cli_gpt2_cpu(tmp_path):
    d = str(tmp_path / "gpt2")
    hf = save_hf_model("gpt2", d, vocab=101, with_tokenizer=True)
    from transformers import AutoTokenizer

    tok = AutoTokenizer.from_pretrained(d)
    prompts = ["hello world", "this is a tiny"]
    for cache in ([], ["--use_cache"]):
        r = subprocess.run([sys.executable, "generate.py", "--pretrained_model_path", d, "--prompts", *prompts,
                            "--max_new_tokens", "6", "--is_greedy", "--device", "cpu", *cache],
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        lines = r.stdout.strip().splitlines()
        assert lines[0].startswith("elapsed time: ") and lines[1] == f"prompts: {prompts}"
        conts = eval(lines[2][len("continuations: "):])
        for p, c in zip(prompts, conts):
            ids = tok(p, return_tensors="pt")["input_ids"]
            with torch.no_grad():
                ref = hf.generate(ids, max_new_tokens=6, do_sample=False, pad_token_id=0)[0, ids.shape[1]:]
            eos = tok.eos_token_id
            ref = ref.tolist()
            if eos in ref:
                ref = ref[:ref.index(eos) + 1]
            assert c == tok.decode(ref)
    # validation identical to the reference
    r = subprocess.run([sys.executable, "generate.py", "--pretrained_model_path", d, "--prompts", "x",
                        "--temperature", "1.5"], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "temperature is not valid" in r.stderr
