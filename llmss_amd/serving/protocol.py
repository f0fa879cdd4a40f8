"""Wire formats (API-compatible with the reference PoC).

HTTP/Redis request JSON = ``{"prompt", "max_new_tokens", "is_greedy", "temperature", "top_p",
"top_k"}`` (producer_server.py:9-15), optionally ``"request_id"``; response JSON =
``{"prompt", "continuation"}`` written with ``ensure_ascii=False`` (consumer_server.py:170-173),
plus ``"request_id"`` and metrics when the request carried an id. Unknown keys are ignored, so a
reference producer/consumer interoperates with ours.
"""
from __future__ import annotations

import json
import uuid
from typing import Any, Dict, List, Optional

from pydantic import BaseModel

from ..engine.sampling import SamplingParams


class Request(BaseModel):
    prompt: str
    max_new_tokens: int = 20
    is_greedy: bool = False
    temperature: float = 1.0
    top_p: float = 0.95
    top_k: int = 50
    request_id: Optional[str] = None
    seed: Optional[int] = None
    # extensions (absent from reference requests; a reference consumer ignores them)
    ignore_eos: bool = False
    stream: bool = False  # reply per engine step on squeue:<request_id>, then a final "finished" message
    prompt_token_ids: Optional[List[int]] = None  # pre-tokenized prompt (prompt text ignored)
    deadline_s: Optional[float] = None  # seconds the caller waits for the reply: the consumer stops generating then


class Response(BaseModel):
    prompt: str
    continuation: str
    request_id: Optional[str] = None
    output_tokens: Optional[int] = None
    ttft_s: Optional[float] = None
    e2e_s: Optional[float] = None
    finish_reason: Optional[str] = None


def new_request_id() -> str:
    return uuid.uuid4().hex


def parse_request(msg: str) -> Request:
    d = json.loads(msg)
    known = {k: d[k] for k in Request.model_fields if k in d}
    return Request(**known)


def to_sampling(req: Request) -> SamplingParams:
    return SamplingParams(max_new_tokens=req.max_new_tokens, is_greedy=req.is_greedy, temperature=req.temperature,
                          top_p=req.top_p, top_k=req.top_k, seed=req.seed, ignore_eos=req.ignore_eos).validate()


def dump_response(resp: Dict[str, Any]) -> str:
    return json.dumps({k: v for k, v in resp.items() if v is not None}, ensure_ascii=False)
