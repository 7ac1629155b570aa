"""Real gRPC server for the ``comfy_request.v1.Comfy`` and ``grpc.health.v1.Health`` services.

The reference ships only protoc output for these contracts and never registers a servicer
(``autogen_python/comfy_request.v1_pb2_grpc.py:9-260``). There is no protoc here, so
the message and service descriptors are built at import time from a ``FileDescriptorProto``
written out below (same package, message names, field numbers, field types and enum values as
the reference contract -> wire compatible with clients generated from the original .proto).
``SerializedGraph`` (from ``serialized_graph.v1``) is carried as opaque bytes, which is
wire-identical for a length-delimited embedded message; it is accepted and ignored.

Handlers share the job model of the HTTP/JSON form in ``service.py`` (one JobTracker):
  Run(ComfyRequest) -> JobSnapshot             GetJob(JobId) -> JobSnapshot
  RunSync(ComfyRequest) -> stream JobOutput    GetNodeDefinitions(NodeDefRequest) -> NodeDefs
  GetModelCatalog(ModelCatalogRequest) -> ModelCatalog
  SyncLocalFiles(google.protobuf.Empty) -> stream LocalFiles
  Health.Check / Health.Watch
Start with ``--grpc-port`` (main.py) or ``start_grpc_server(prompt_server, port)``.
"""
from __future__ import annotations

import concurrent.futures
import logging
import time

from google.protobuf import descriptor_pb2, descriptor_pool, empty_pb2, json_format, message_factory, struct_pb2

F = descriptor_pb2.FieldDescriptorProto
_T = {"string": F.TYPE_STRING, "bool": F.TYPE_BOOL, "int64": F.TYPE_INT64, "uint32": F.TYPE_UINT32,
      "bytes": F.TYPE_BYTES, "enum": F.TYPE_ENUM, "msg": F.TYPE_MESSAGE}

# (message, [(field, number, type, label, type_name, oneof_index)], nested, oneofs, options)
_PKG = "comfy_request.v1"


def _field(name, num, typ, rep=False, type_name=None, oneof=None, proto3_optional=False):
    f = F(name=name, number=num, type=_T[typ], label=F.LABEL_REPEATED if rep else F.LABEL_OPTIONAL)
    if type_name:
        f.type_name = type_name
    if oneof is not None:
        f.oneof_index = oneof
    if proto3_optional:
        f.proto3_optional = True
    f.json_name = "".join(w.capitalize() if i else w for i, w in enumerate(name.split("_")))
    return f


def _msg(name, fields, nested=(), oneofs=(), map_entry=False):
    m = descriptor_pb2.DescriptorProto(name=name)
    m.field.extend(fields)
    m.nested_type.extend(nested)
    for o in oneofs:
        m.oneof_decl.add(name=o)
    if map_entry:
        m.options.map_entry = True
    return m


def _map_entry(name, value_type):
    return _msg(name, [_field("key", 1, "string"), _field("value", 2, "msg", type_name=value_type)], map_entry=True)


def _build_file():
    p = f".{_PKG}."
    fd = descriptor_pb2.FileDescriptorProto(name="cgs_comfy_request.v1.proto", package=_PKG, syntax="proto3")
    fd.dependency.extend(["google/protobuf/struct.proto", "google/protobuf/empty.proto"])
    fd.enum_type.add(name="JobStatus").value.extend([
        descriptor_pb2.EnumValueDescriptorProto(name=n, number=i)
        for i, n in enumerate(["QUEUED", "EXECUTING", "COMPLETED", "ERROR", "ABORTED"])])
    fd.message_type.extend([
        _msg("WorkflowStep", [_field("class_type", 1, "string"),
                              _field("inputs", 2, "msg", type_name=".google.protobuf.Struct")]),
        _msg("FileReference", [_field("url", 1, "string"), _field("is_temp", 2, "bool")]),
        _msg("WorkflowFile", [_field("blake3_hash", 1, "string"), _field("mime_type", 2, "string"),
                              _field("reference", 3, "msg", type_name=p + "FileReference", oneof=0),
                              _field("bytes", 4, "bytes", oneof=0)], oneofs=["data"]),
        _msg("LocalFile", [_field("name", 1, "string"), _field("path", 2, "string"), _field("size", 3, "int64"),
                           _field("mime_type", 4, "string")]),
        _msg("LocalFiles", [_field(n, i + 1, "msg", rep=True, type_name=p + "LocalFile")
                            for i, n in enumerate(["added", "updated", "removed"])]),
        _msg("JobId", [_field("job_id", 1, "string")]),
        _msg("OutputConfig", [_field("write_to_graph_id", 1, "string", oneof=0, proto3_optional=True),
                              _field("webhook_url", 2, "string", oneof=1, proto3_optional=True)],
             oneofs=["_write_to_graph_id", "_webhook_url"]),
        _msg("ComfyRequest", [_field("request_id", 1, "string", oneof=0, proto3_optional=True),
                              _field("workflow", 2, "msg", rep=True, type_name=p + "ComfyRequest.WorkflowEntry"),
                              _field("serialized_graph", 3, "bytes", oneof=1, proto3_optional=True),
                              _field("output_config", 4, "msg", type_name=p + "OutputConfig", oneof=2,
                                     proto3_optional=True)],
             nested=[_map_entry("WorkflowEntry", p + "WorkflowStep")],
             oneofs=["_request_id", "_serialized_graph", "_output_config"]),
        _msg("JobSnapshot", [_field("job_id", 1, "string"),
                             _field("request_id", 2, "string", oneof=0, proto3_optional=True),
                             _field("status", 3, "enum", type_name=p + "JobStatus"),
                             _field("outputs", 4, "msg", rep=True, type_name=p + "JobOutput"),
                             _field("metrics", 5, "msg", type_name=p + "JobSnapshot.Metrics", oneof=1,
                                    proto3_optional=True)],
             nested=[_msg("Metrics", [_field("queue_seconds", 1, "uint32"), _field("execution_seconds", 2, "uint32")])],
             oneofs=["_request_id", "_metrics"]),
        _msg("JobOutput", [_field("node_id", 1, "string"), _field("class_type", 2, "string"),
                           _field("file", 3, "msg", type_name=p + "WorkflowFile")]),
        _msg("NodeDefRequest", [_field("extension_ids", 1, "string", rep=True)]),
        _msg("NodeDefinition", [_field("display_name", 1, "string"), _field("description", 2, "string"),
                                _field("category", 3, "string"),
                                _field("inputs", 4, "msg", rep=True, type_name=p + "NodeDefinition.InputDef"),
                                _field("outputs", 5, "msg", rep=True, type_name=p + "NodeDefinition.OutputDef"),
                                _field("output_node", 6, "bool")],
             nested=[_msg("InputDef", [_field("label", 1, "string"), _field("edge_type", 2, "string"),
                                       _field("spec", 3, "msg", type_name=".google.protobuf.Struct")]),
                     _msg("OutputDef", [_field("label", 1, "string"), _field("edge_type", 2, "string")])]),
        _msg("NodeDefs", [_field("defs", 1, "msg", rep=True, type_name=p + "NodeDefs.DefsEntry")],
             nested=[_map_entry("DefsEntry", p + "NodeDefinition")]),
        _msg("Models", [_field("info", 1, "msg", rep=True, type_name=p + "Models.Info")],
             nested=[_msg("Info", [_field("blake3_hash", 1, "string"), _field("display_name", 2, "string")])]),
        _msg("ModelCatalog", [_field("models", 1, "msg", rep=True, type_name=p + "ModelCatalog.ModelsEntry")],
             nested=[_map_entry("ModelsEntry", p + "Models")]),
        _msg("ModelCatalogRequest", [_field("base_family", 1, "string", rep=True)]),
    ])
    svc = fd.service.add(name="Comfy")
    for name, req, resp, stream in [("Run", "ComfyRequest", "JobSnapshot", False),
                                    ("RunSync", "ComfyRequest", "JobOutput", True),
                                    ("GetJob", "JobId", "JobSnapshot", False),
                                    ("GetNodeDefinitions", "NodeDefRequest", "NodeDefs", False),
                                    ("GetModelCatalog", "ModelCatalogRequest", "ModelCatalog", False),
                                    ("SyncLocalFiles", ".google.protobuf.Empty", "LocalFiles", True)]:
        m = svc.method.add(name=name, input_type=req if req.startswith(".") else p + req, output_type=p + resp)
        m.server_streaming = stream
    return fd


def _build_health():
    fd = descriptor_pb2.FileDescriptorProto(name="cgs_grpc_health_v1.proto", package="grpc.health.v1", syntax="proto3")
    fd.message_type.add(name="HealthCheckRequest").field.extend([_field("service", 1, "string")])
    r = fd.message_type.add(name="HealthCheckResponse")
    e = r.enum_type.add(name="ServingStatus")
    e.value.extend([descriptor_pb2.EnumValueDescriptorProto(name=n, number=i)
                    for i, n in enumerate(["UNKNOWN", "SERVING", "NOT_SERVING", "SERVICE_UNKNOWN"])])
    r.field.extend([_field("status", 1, "enum", type_name=".grpc.health.v1.HealthCheckResponse.ServingStatus")])
    svc = fd.service.add(name="Health")
    svc.method.add(name="Check", input_type=".grpc.health.v1.HealthCheckRequest",
                   output_type=".grpc.health.v1.HealthCheckResponse")
    svc.method.add(name="Watch", input_type=".grpc.health.v1.HealthCheckRequest",
                   output_type=".grpc.health.v1.HealthCheckResponse", server_streaming=True)
    return fd


_POOL = descriptor_pool.DescriptorPool()
for _dep in (struct_pb2, empty_pb2):
    _POOL.Add(descriptor_pb2.FileDescriptorProto.FromString(_dep.DESCRIPTOR.serialized_pb))
_POOL.Add(_build_file())
_POOL.Add(_build_health())


def message_class(full_name):
    return message_factory.GetMessageClass(_POOL.FindMessageTypeByName(full_name))


M = {n: message_class(f"{_PKG}.{n}") for n in
     ("ComfyRequest", "JobSnapshot", "JobOutput", "JobId", "NodeDefRequest", "NodeDefs", "ModelCatalogRequest",
      "ModelCatalog", "LocalFiles", "WorkflowStep")}
HealthCheckRequest = message_class("grpc.health.v1.HealthCheckRequest")
HealthCheckResponse = message_class("grpc.health.v1.HealthCheckResponse")
Empty = message_class("google.protobuf.Empty")
TERMINAL = (2, 3, 4)   # COMPLETED, ERROR, ABORTED


def _from_dict(cls, d):
    msg = cls()
    json_format.ParseDict(d, msg, ignore_unknown_fields=True)
    return msg


def _request_to_dict(req):
    d = json_format.MessageToDict(req, preserving_proto_field_name=True)
    d.pop("serialized_graph", None)
    return d


class ComfyServicer:
    def __init__(self, prompt_server):
        from . import service
        self.server = prompt_server
        self.service = service
        self.tracker = getattr(prompt_server, "job_tracker", None) or service.JobTracker(prompt_server)
        prompt_server.job_tracker = self.tracker

    def _snapshot(self, job_id, context=None):
        snap = self.tracker.snapshot(job_id)
        if snap["status"] < 0 and context is not None:
            import grpc
            context.abort(grpc.StatusCode.NOT_FOUND, f"unknown job {job_id}")
        snap = dict(snap)
        snap.pop("status_name", None)
        if snap["status"] < 0:
            snap["status"] = 0
        return _from_dict(M["JobSnapshot"], snap)

    def Run(self, request, context):
        import grpc
        job_id, err = self.service.submit_request(self.server, self.tracker, _request_to_dict(request))
        if err is not None:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(err.get("error", err))[:2000])
        return self._snapshot(job_id)

    def RunSync(self, request, context):
        import grpc
        job_id, err = self.service.submit_request(self.server, self.tracker, _request_to_dict(request))
        if err is not None:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(err.get("error", err))[:2000])
        sent = 0
        while context.is_active():
            snap = self.tracker.snapshot(job_id)
            for o in snap["outputs"][sent:]:
                yield _from_dict(M["JobOutput"], o)
            sent = len(snap["outputs"])
            if snap["status"] in TERMINAL:
                return
            time.sleep(0.05)

    def GetJob(self, request, context):
        return self._snapshot(request.job_id, context)

    def GetNodeDefinitions(self, request, context):
        return _from_dict(M["NodeDefs"], {"defs": self.service.node_definitions(list(request.extension_ids))})

    def GetModelCatalog(self, request, context):
        return _from_dict(M["ModelCatalog"], {"models": self.service.model_catalog(list(request.base_family))})

    def SyncLocalFiles(self, request, context):
        yield _from_dict(M["LocalFiles"], self.service.local_files_delta(self.tracker))


def _handlers(servicer):
    import grpc
    u, s = grpc.unary_unary_rpc_method_handler, grpc.unary_stream_rpc_method_handler
    ser = lambda m: m.SerializeToString()  # noqa: E731
    comfy = grpc.method_handlers_generic_handler(f"{_PKG}.Comfy", {
        "Run": u(servicer.Run, M["ComfyRequest"].FromString, ser),
        "RunSync": s(servicer.RunSync, M["ComfyRequest"].FromString, ser),
        "GetJob": u(servicer.GetJob, M["JobId"].FromString, ser),
        "GetNodeDefinitions": u(servicer.GetNodeDefinitions, M["NodeDefRequest"].FromString, ser),
        "GetModelCatalog": u(servicer.GetModelCatalog, M["ModelCatalogRequest"].FromString, ser),
        "SyncLocalFiles": s(servicer.SyncLocalFiles, Empty.FromString, ser),
    })

    def check(req, ctx):
        return HealthCheckResponse(status=1)

    def watch(req, ctx):
        while ctx.is_active():
            yield HealthCheckResponse(status=1)
            time.sleep(1.0)

    health = grpc.method_handlers_generic_handler("grpc.health.v1.Health", {
        "Check": u(check, HealthCheckRequest.FromString, ser),
        "Watch": s(watch, HealthCheckRequest.FromString, ser),
    })
    return [comfy, health]


def start_grpc_server(prompt_server, port=50051, host="0.0.0.0", workers=8):
    import grpc
    srv = grpc.server(concurrent.futures.ThreadPoolExecutor(max_workers=workers))
    srv.add_generic_rpc_handlers(_handlers(ComfyServicer(prompt_server)))
    bound = srv.add_insecure_port(f"{host}:{port}")
    srv.start()
    logging.info("gRPC comfy_request.v1.Comfy + grpc.health.v1.Health on %s:%d", host, bound)
    return srv, bound


def stubs(channel):
    """Client-side callables (for tests / tools): name -> multi-callable."""
    ser = lambda m: m.SerializeToString()  # noqa: E731
    out = {}
    for name, req, resp, stream in [("Run", "ComfyRequest", "JobSnapshot", False),
                                    ("RunSync", "ComfyRequest", "JobOutput", True),
                                    ("GetJob", "JobId", "JobSnapshot", False),
                                    ("GetNodeDefinitions", "NodeDefRequest", "NodeDefs", False),
                                    ("GetModelCatalog", "ModelCatalogRequest", "ModelCatalog", False)]:
        mk = channel.unary_stream if stream else channel.unary_unary
        out[name] = mk(f"/{_PKG}.Comfy/{name}", request_serializer=ser, response_deserializer=M[resp].FromString)
    out["SyncLocalFiles"] = channel.unary_stream(f"/{_PKG}.Comfy/SyncLocalFiles", request_serializer=ser,
                                                 response_deserializer=M["LocalFiles"].FromString)
    out["Check"] = channel.unary_unary("/grpc.health.v1.Health/Check", request_serializer=ser,
                                       response_deserializer=HealthCheckResponse.FromString)
    return out
