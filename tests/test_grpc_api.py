"""vLLM gRPC engine API (vllm.grpc.engine.VllmEngine, docs/api-reference/
epp-grpc-apis.md) end to end on CPU: the engine's gRPC server (Generate
unary-complete and streaming, Embed), and the same calls through the router's
gRPC data plane with the EPP's vllmgrpc-parser (protobuf frames parsed for
routing and prefix scoring, usage accounted from the response frames, EPP
rejections as gRPC status codes)."""
import asyncio

import aiohttp
import grpc
import pytest
from aiohttp import web

from llmd_amd.engine.config import EngineConfig
from llmd_amd.router.api import ControlPlane
from llmd_amd.router.datalayer import EndpointStore, endpoints_from_yaml
from llmd_amd.router.epp import EPP
from llmd_amd.router.grpc_proxy import GrpcRouter
from llmd_amd.serving import vllm_grpc as vg
from llmd_amd.serving.api_server import build_server

CONF = """
apiVersion: llm-d.ai/v1alpha1
kind: EndpointPickerConfig
plugins:
- type: vllmgrpc-parser
- type: prefix-cache-scorer
- type: queue-scorer
- type: max-score-picker
schedulingProfiles:
- name: default
  plugins:
  - pluginRef: prefix-cache-scorer
    weight: 3
  - pluginRef: queue-scorer
    weight: 1
  - pluginRef: max-score-picker
requestHandler:
  parsers:
  - pluginRef: vllmgrpc-parser
"""


def _cfg():
    return EngineConfig.create("tiny-llama", device="cpu", block_size=16, num_gpu_blocks=64,
                               max_num_batched_tokens=128, max_num_seqs=4, max_model_len=512, enforce_eager=True)


async def _serve(app):
    runner = web.AppRunner(app, access_log=None)
    await runner.setup()
    site = web.TCPSite(runner, "127.0.0.1", 0)
    await site.start()
    return runner, site._server.sockets[0].getsockname()[1]


def test_engine_grpc_and_router_data_plane():
    ids = [5, 6, 7, 8, 9, 10, 11]

    async def main():
        srv = build_server(_cfg())
        runner, http_port = await _serve(srv.app())
        gsrv, gport = await vg.start_server(srv, 0, "127.0.0.1")
        out = {}
        try:
            c = vg.Client(f"127.0.0.1:{gport}")
            out["unary"], _ = await c.generate(input_ids=ids, max_tokens=6, ignore_eos=True)
            out["stream"], _ = await c.generate(input_ids=ids, max_tokens=6, ignore_eos=True, stream=True)
            out["emb"] = await c.embed(ids)
            out["text"], _ = await c.generate(text="hello world", max_tokens=3, ignore_eos=True)
            try:
                await c.generate(input_ids=[10 ** 7], max_tokens=2)
            except grpc.aio.AioRpcError as e:
                out["bad"] = e.code()
            await c.close()
            async with aiohttp.ClientSession() as s:
                async with s.post(f"http://127.0.0.1:{http_port}/inference/v1/generate", json={
                        "token_ids": ids, "sampling_params": {"max_tokens": 6, "temperature": 0,
                                                              "ignore_eos": True}}) as r:
                    out["http"] = (await r.json())["choices"][0]["token_ids"]
            # ---- through the router: EPP (vllmgrpc-parser) + gRPC data plane
            store = EndpointStore()
            for e in endpoints_from_yaml({"endpoints": [{"name": "e0", "address": "127.0.0.1",
                                                         "port": http_port}]}):
                await store.add(e)
            epp = EPP(CONF, store, ControlPlane(), "pool")
            await epp.start()
            gr = GrpcRouter(epp, lambda key: f"127.0.0.1:{gport}")
            rport = await gr.start(0, "127.0.0.1")
            rc = vg.Client(f"127.0.0.1:{rport}")
            md = (("x-llm-d-inference-fairness-id", "tenant-a"), ("x-request-id", "grpc-r1"))
            out["r_unary"], _ = await rc.generate(input_ids=ids, max_tokens=6, ignore_eos=True, metadata=md)
            out["r_stream"], _ = await rc.generate(input_ids=ids, max_tokens=6, ignore_eos=True, stream=True)
            out["r_emb"] = await rc.embed(ids)
            await rc.close()
            out["metrics"] = epp.render_metrics().decode()
            out["epp_parsed"] = epp.parse(vg.GENERATE, vg.frame(vg.PB["GenerateRequest"](
                request_id="x", tokenized=vg.PB["TokenizedInput"](input_ids=ids), stream=True).SerializeToString()),
                {})
            await gr.stop()
            await epp.stop()
        finally:
            await gsrv.stop(grace=0.5)
            await runner.cleanup()
            srv.aeng.shutdown()
        return out

    out = asyncio.run(main())
    (u,) = out["unary"]
    assert u.WhichOneof("response") == "complete"
    assert list(u.complete.output_ids) == out["http"]
    assert u.complete.prompt_tokens == len(ids) and u.complete.completion_tokens == 6
    assert u.complete.finish_reason == "length"
    st = out["stream"]
    assert [m.WhichOneof("response") for m in st][-1] == "complete"
    assert [t for m in st[:-1] for t in m.chunk.token_ids] == out["http"]
    assert st[-1].complete.completion_tokens == 6 and not st[-1].complete.output_ids
    assert out["emb"].embedding_dim == len(out["emb"].embedding) > 0 and out["emb"].prompt_tokens == len(ids)
    assert out["text"][-1].complete.completion_tokens == 3
    assert out["bad"] == grpc.StatusCode.INVALID_ARGUMENT
    # routed calls return the same tokens
    assert list(out["r_unary"][0].complete.output_ids) == out["http"]
    assert [t for m in out["r_stream"][:-1] for t in m.chunk.token_ids] == out["http"]
    assert list(out["r_emb"].embedding) == list(out["emb"].embedding)
    p = out["epp_parsed"]
    assert p.token_ids == ids and p.stream and p.data.get("grpc") and p.request_id == "x"
    m = out["metrics"]
    assert "inference_objective_request_total" in m and "scheduler_attempts_total" in m


def test_grpc_parser_rejects_bad_frames():
    from llmd_amd.router.plugins.parsers import VllmGrpcParser

    p = VllmGrpcParser("vllmgrpc-parser", {})
    with pytest.raises(ValueError):
        p.parse(vg.GENERATE, b"\x00\x00\x00\x00\x05abc", {})  # truncated frame: no message
    with pytest.raises(ValueError):
        p.parse(vg.GENERATE, vg.frame(b"\xff\xff\xff"), {})
    # the JSON token-in bridge keeps working
    r = p.parse("/inference/v1/generate", b'{"token_ids": [1, 2, 3]}', {})
    assert r.token_ids == [1, 2, 3]
