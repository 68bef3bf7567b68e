"""The ``gpu_sim`` wire schema, built programmatically (no protoc / grpc_tools in
this image).

Wire compatibility with the reference: package ``gpu_sim``, services
``gpu_sim.GPUDevice`` / ``gpu_sim.GPUCoordinator``, every message / enum /
field name and field number of ``DSML/proto/gpu_sim.proto``, so a
reference client can talk to these servers.  Additions only use NEW field
numbers and NEW methods:

* ``RunForward`` / ``RunBackward`` — present only in the reference's stale
  generated code (``gpu_sim.pb.go:1225-1425``); implemented here.
* ``AllReduceRingRequest.dtype`` (5), ``algo`` (6): dtype-aware reduction
  instead of the reference's byte-wise uint8 add.
* ``CommInitRequest.backend`` (3): ``"rpc"`` moves data device->device over
  gRPC streams; ``"rccl"`` bootstraps an RCCL communicator on the device GPUs;
  ``"pg"`` bootstraps a torch.distributed process group on the device servers
  over a TCP store the coordinator hosts (``CommSetupRequest.storeAddress``, 6),
  plus an RCCL communicator when every device owns a distinct GPU: data-parallel
  ``TrainSteps`` then runs the fused xGMI / persistent data-parallel steps
  (every candidate self-tested and timed, the fastest kept).
* ``BeginSendRequest.dstAddress`` (4), ``DataChunk.srcRank`` (3): the device
  pushes the data itself (the proto comment's intended semantics,
  ``gpu_sim.proto:32-34``) instead of the coordinator relaying it.
* GPUDevice: Reduce, GetCommUniqueId, CommSetup, DeviceAllReduce, Abort,
  CommTeardown, ConfigureModel, TrainSteps, Evaluate, ApplyGradients, GetStats.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

PACKAGE = "gpu_sim"
FD = descriptor_pb2.FieldDescriptorProto

_SCALARS = {
    "uint64": FD.TYPE_UINT64, "uint32": FD.TYPE_UINT32, "int64": FD.TYPE_INT64,
    "int32": FD.TYPE_INT32, "bool": FD.TYPE_BOOL, "bytes": FD.TYPE_BYTES,
    "string": FD.TYPE_STRING, "double": FD.TYPE_DOUBLE, "float": FD.TYPE_FLOAT,
}

# Enums: name -> [(value_name, number)]
ENUMS: Dict[str, List[Tuple[str, int]]] = {
    "Status": [("IN_PROGRESS", 0), ("SUCCESS", 1), ("FAILED", 2)],
    "ReduceOp": [("SUM", 0), ("PROD", 1), ("MIN", 2), ("MAX", 3)],
    # extension: element type of an all-reduce / reduce (default FLOAT32)
    "DataType": [("FLOAT32", 0), ("UINT8", 1), ("BFLOAT16", 2), ("FLOAT16", 3), ("INT32", 4)],
}

# Messages: name -> [(field, number, type, label)] ; label "" | "repeated" | "oneof:<name>" | "map:<k>:<v>"
M = Dict[str, List[Tuple]]
MESSAGES: M = {
    # -- ids -------------------------------------------------------------
    "DeviceId": [("value", 1, "uint64")],
    "Rank": [("value", 1, "uint32")],
    "MemAddr": [("value", 1, "uint64")],
    "StreamId": [("value", 1, "uint64")],
    "DeviceMetadata": [("deviceId", 1, ".DeviceId"), ("minMemAddr", 2, ".MemAddr"),
                       ("maxMemAddr", 3, ".MemAddr"),
                       # extension
                       ("name", 4, "string"), ("backend", 5, "string"),
                       ("host", 6, "string")],  # the server's hostname (node identity)
    # -- device ------------------------------------------------------------
    "GetDeviceMetadataRequest": [],
    "GetDeviceMetadataResponse": [("metadata", 1, ".DeviceMetadata")],
    "BeginSendRequest": [("sendBuffAddr", 1, ".MemAddr"), ("numBytes", 2, "uint64"),
                         ("dstRank", 3, ".Rank"), ("dstAddress", 4, "string")],
    "BeginSendResponse": [("initiated", 1, "bool"), ("streamId", 2, ".StreamId")],
    "BeginReceiveRequest": [("streamId", 1, ".StreamId"), ("recvBuffAddr", 2, ".MemAddr"),
                            ("numBytes", 3, "uint64"), ("srcRank", 4, ".Rank")],
    "BeginReceiveResponse": [("initiated", 1, "bool")],
    "DataChunk": [("data", 1, "bytes"), ("streamId", 2, "uint64"), ("srcRank", 3, "uint32")],
    "StreamSendResponse": [("success", 1, "bool")],
    # device-driven ring over ONE long-lived client stream per neighbour pair
    # (GPUDevice.RingChannel): every ring step of every call is one message
    "RingChunk": [("commId", 1, "uint64"), ("seq", 2, "uint64"), ("step", 3, "uint32"),
                  ("srcRank", 4, "uint32"), ("data", 5, "bytes")],
    "RingAck": [("success", 1, "bool")],
    "GetStreamStatusRequest": [("streamId", 1, ".StreamId")],
    "GetStreamStatusResponse": [("status", 1, ".Status")],
    # -- memcpy ------------------------------------------------------------
    "MemcpyHostToDeviceRequest": [("hostSrcData", 1, "bytes"), ("dstDeviceId", 2, ".DeviceId"),
                                  ("dstMemAddr", 3, ".MemAddr")],
    "MemcpyHostToDeviceResponse": [("success", 1, "bool")],
    "MemcpyDeviceToHostRequest": [("srcDeviceId", 1, ".DeviceId"), ("srcMemAddr", 2, ".MemAddr"),
                                  ("numBytes", 3, "uint64")],
    "MemcpyDeviceToHostResponse": [("dstData", 1, "bytes")],
    "MemcpyRequest": [("hostToDevice", 1, ".MemcpyHostToDeviceRequest", "oneof:either"),
                      ("deviceToHost", 2, ".MemcpyDeviceToHostRequest", "oneof:either")],
    "MemcpyResponse": [("hostToDevice", 1, ".MemcpyHostToDeviceResponse", "oneof:either"),
                       ("deviceToHost", 2, ".MemcpyDeviceToHostResponse", "oneof:either")],
    # -- coordinator -------------------------------------------------------
    "CommInitRequest": [("numDevices", 1, "uint32"), ("device_addresses", 2, "string", "repeated"),
                        ("backend", 3, "string")],
    "CommInitResponse": [("success", 1, "bool"), ("commId", 2, "uint64"),
                         ("devices", 3, ".DeviceMetadata", "repeated")],
    "GetCommStatusRequest": [("commId", 1, "uint64"), ("device_addresses", 2, "string", "repeated")],
    "GetCommStatusResponse": [("status", 1, ".Status"), ("error", 2, "string")],
    "GroupStartRequest": [("commId", 1, "uint64")],
    "GroupStartResponse": [("success", 1, "bool")],
    "GroupEndRequest": [("commId", 1, "uint64")],
    "GroupEndResponse": [("success", 1, "bool")],
    "AllReduceRingRequest": [("commId", 1, "uint64"), ("count", 2, "uint64"), ("op", 3, ".ReduceOp"),
                             ("memAddrs", 4, "", "map:uint32:.MemAddr"),
                             ("dtype", 5, ".DataType"), ("algo", 6, "string"),
                             ("chunkBytes", 7, "uint64")],
    "AllReduceRingResponse": [("success", 1, "bool"), ("elapsedUs", 2, "double"),
                              ("algo", 3, "string"), ("chunkBytes", 4, "uint64")],  # what ran
    "CommDestroyRequest": [("commId", 1, "uint64")],
    "CommDestroyResponse": [("success", 1, "bool")],
    "CommFinalizeRequest": [("commId", 1, "uint64")],
    "CommFinalizeResponse": [("success", 1, "bool")],
    "NaiveAllReduceRequest": [("commId", 1, "uint64"), ("dataSize", 2, "uint64"),
                              ("latencyMs", 3, "uint32")],
    "NaiveAllReduceResponse": [("success", 1, "bool"), ("totalTimeMs", 2, "int64"),
                               ("totalDataTransferred", 3, "int64"),
                               ("totalTimeUs", 4, "double")],
    # -- stale-generated RunForward / RunBackward (gpu_sim.pb.go:1225-1425) --
    "RunForwardRequest": [("deviceId", 1, "uint64"), ("inputAddr", 2, "uint64"),
                          ("outputAddr", 3, "uint64"),
                          ("numRows", 4, "uint32"), ("labelsAddr", 5, "uint64")],
    "RunForwardResponse": [("success", 1, "bool"), ("loss", 2, "double"), ("correct", 3, "uint32")],
    "RunBackwardRequest": [("deviceId", 1, "uint64"), ("gradientAddr", 2, "uint64")],
    "RunBackwardResponse": [("success", 1, "bool"), ("numBytes", 2, "uint64")],
    # -- extensions (device) -------------------------------------------------
    "ReduceRequest": [("dstAddr", 1, "uint64"), ("srcAddr", 2, "uint64"), ("numBytes", 3, "uint64"),
                      ("dtype", 4, ".DataType"), ("op", 5, ".ReduceOp"), ("scale", 6, "double"),
                      ("waitStreamId", 7, "uint64")],
    "WaitStreamRequest": [("streamId", 1, ".StreamId"), ("timeoutMs", 2, "uint32")],
    "WaitStreamResponse": [("status", 1, ".Status")],
    "ReduceResponse": [("success", 1, "bool")],
    "GetCommUniqueIdRequest": [("commId", 1, "uint64")],
    "GetCommUniqueIdResponse": [("uniqueId", 1, "bytes")],
    "CommSetupRequest": [("commId", 1, "uint64"), ("uniqueId", 2, "bytes"), ("rank", 3, "uint32"),
                         ("nranks", 4, "uint32"), ("peerAddresses", 5, "string", "repeated"),
                         ("storeAddress", 6, "string")],
    "CommSetupResponse": [("success", 1, "bool"), ("backend", 2, "string")],
    "DeviceAllReduceRequest": [("commId", 1, "uint64"), ("addr", 2, "uint64"), ("count", 3, "uint64"),
                               ("dtype", 4, ".DataType"), ("op", 5, ".ReduceOp"),
                               ("algo", 6, "string"), ("chunkBytes", 7, "uint64"),
                               ("repeat", 8, "uint32")],
    "DeviceAllReduceResponse": [("success", 1, "bool"), ("elapsedUs", 2, "double"),
                                ("algo", 3, "string"), ("chunkBytes", 4, "uint64")],
    "AbortRequest": [("commId", 1, "uint64"), ("reason", 2, "string")],
    "AbortResponse": [("success", 1, "bool")],
    "CommTeardownRequest": [("commId", 1, "uint64")],
    "CommTeardownResponse": [("success", 1, "bool")],
    "ConfigureModelRequest": [("dims", 1, "uint32", "repeated"), ("batch", 2, "uint32"),
                              ("lr", 3, "double"), ("seed", 4, "uint64"), ("commId", 5, "uint64"),
                              ("rank", 6, "uint32"), ("worldSize", 7, "uint32"),
                              ("dataset", 8, "string"), ("numSamples", 9, "uint64"),
                              ("weightsAddr", 10, "uint64"), ("momentum", 11, "double"),
                              ("graphSteps", 12, "uint32"), ("sync", 13, "string"),
                              ("dataSeed", 14, "uint64")],
    "ConfigureModelResponse": [("success", 1, "bool"), ("numParams", 2, "uint64"),
                               ("batchesPerEpoch", 3, "uint64"), ("paramBytes", 4, "uint64"),
                               ("sync", 5, "string"), ("syncTimesJson", 6, "string")],
    "TrainStepsRequest": [("steps", 1, "uint64")],
    "TrainStepsResponse": [("success", 1, "bool"), ("lossSum", 2, "double"), ("correct", 3, "double"),
                           ("count", 4, "double"), ("elapsedUs", 5, "double"),
                           ("stepsDone", 6, "uint64")],
    "EvaluateRequest": [("dataset", 1, "string"), ("numSamples", 2, "uint64"), ("seed", 3, "uint64")],
    "EvaluateResponse": [("success", 1, "bool"), ("accuracy", 2, "double"), ("loss", 3, "double"),
                         ("count", 4, "uint64")],
    "ApplyGradientsRequest": [("gradientAddr", 1, "uint64"), ("scale", 2, "double")],
    "ApplyGradientsResponse": [("success", 1, "bool")],
    "GetStatsRequest": [],
    "GetStatsResponse": [("json", 1, "string")],
}

# Services: name -> [(method, request, response, client_streaming)]
SERVICES = {
    "GPUDevice": [
        ("GetDeviceMetadata", "GetDeviceMetadataRequest", "GetDeviceMetadataResponse", False),
        ("BeginSend", "BeginSendRequest", "BeginSendResponse", False),
        ("BeginReceive", "BeginReceiveRequest", "BeginReceiveResponse", False),
        ("StreamSend", "DataChunk", "StreamSendResponse", True),
        ("RingChannel", "RingChunk", "RingAck", True),
        ("GetStreamStatus", "GetStreamStatusRequest", "GetStreamStatusResponse", False),
        ("Memcpy", "MemcpyRequest", "MemcpyResponse", False),
        ("RunForward", "RunForwardRequest", "RunForwardResponse", False),
        ("RunBackward", "RunBackwardRequest", "RunBackwardResponse", False),
        ("Reduce", "ReduceRequest", "ReduceResponse", False),
        ("WaitStream", "WaitStreamRequest", "WaitStreamResponse", False),
        ("GetCommUniqueId", "GetCommUniqueIdRequest", "GetCommUniqueIdResponse", False),
        ("CommSetup", "CommSetupRequest", "CommSetupResponse", False),
        ("DeviceAllReduce", "DeviceAllReduceRequest", "DeviceAllReduceResponse", False),
        ("Abort", "AbortRequest", "AbortResponse", False),
        ("CommTeardown", "CommTeardownRequest", "CommTeardownResponse", False),
        ("ConfigureModel", "ConfigureModelRequest", "ConfigureModelResponse", False),
        ("TrainSteps", "TrainStepsRequest", "TrainStepsResponse", False),
        ("Evaluate", "EvaluateRequest", "EvaluateResponse", False),
        ("ApplyGradients", "ApplyGradientsRequest", "ApplyGradientsResponse", False),
        ("GetStats", "GetStatsRequest", "GetStatsResponse", False),
    ],
    "GPUCoordinator": [
        ("CommInit", "CommInitRequest", "CommInitResponse", False),
        ("GetCommStatus", "GetCommStatusRequest", "GetCommStatusResponse", False),
        ("CommDestroy", "CommDestroyRequest", "CommDestroyResponse", False),
        ("CommFinalize", "CommFinalizeRequest", "CommFinalizeResponse", False),
        ("GroupStart", "GroupStartRequest", "GroupStartResponse", False),
        ("GroupEnd", "GroupEndRequest", "GroupEndResponse", False),
        ("AllReduceRing", "AllReduceRingRequest", "AllReduceRingResponse", False),
        ("NaiveAllReduce", "NaiveAllReduceRequest", "NaiveAllReduceResponse", False),
        ("Memcpy", "MemcpyRequest", "MemcpyResponse", False),
    ],
}


def _type_ref(t: str) -> str:
    return f".{PACKAGE}{t}" if t.startswith(".") else t


def _add_field(msg, name, number, typ, label=""):
    f = msg.field.add()
    f.name = name
    f.number = number
    f.json_name = name
    if label == "repeated":
        f.label = FD.LABEL_REPEATED
    else:
        f.label = FD.LABEL_OPTIONAL
    if typ in _SCALARS:
        f.type = _SCALARS[typ]
    else:
        enum_name = typ.lstrip(".")
        f.type = FD.TYPE_ENUM if enum_name in ENUMS else FD.TYPE_MESSAGE
        f.type_name = _type_ref(typ)
    return f


def _build_file() -> descriptor_pb2.FileDescriptorProto:
    fp = descriptor_pb2.FileDescriptorProto()
    fp.name = "hipdsml/gpu_sim.proto"
    fp.package = PACKAGE
    fp.syntax = "proto3"
    for ename, values in ENUMS.items():
        e = fp.enum_type.add()
        e.name = ename
        for vname, num in values:
            v = e.value.add()
            v.name = vname
            v.number = num
    for mname, fields in MESSAGES.items():
        m = fp.message_type.add()
        m.name = mname
        oneofs: Dict[str, int] = {}
        for spec in fields:
            name, number, typ = spec[0], spec[1], spec[2]
            label = spec[3] if len(spec) > 3 else ""
            if label.startswith("map:"):
                _, ktyp, vtyp = label.split(":")
                entry = m.nested_type.add()
                entry.name = name[0].upper() + name[1:] + "Entry"
                entry.options.map_entry = True
                _add_field(entry, "key", 1, ktyp)
                _add_field(entry, "value", 2, vtyp)
                f = m.field.add()
                f.name = name
                f.number = number
                f.json_name = name
                f.label = FD.LABEL_REPEATED
                f.type = FD.TYPE_MESSAGE
                f.type_name = f".{PACKAGE}.{mname}.{entry.name}"
            elif label.startswith("oneof:"):
                oname = label.split(":", 1)[1]
                if oname not in oneofs:
                    oneofs[oname] = len(m.oneof_decl)
                    m.oneof_decl.add().name = oname
                f = _add_field(m, name, number, typ)
                f.oneof_index = oneofs[oname]
            else:
                _add_field(m, name, number, typ, label)
    for sname, methods in SERVICES.items():
        s = fp.service.add()
        s.name = sname
        for meth, req, resp, cstream in methods:
            mm = s.method.add()
            mm.name = meth
            mm.input_type = f".{PACKAGE}.{req}"
            mm.output_type = f".{PACKAGE}.{resp}"
            mm.client_streaming = cstream
    return fp


_pool = descriptor_pool.DescriptorPool()
FILE = _pool.Add(_build_file())


class _Namespace:
    pass


pb = _Namespace()
for _name in MESSAGES:
    setattr(pb, _name, message_factory.GetMessageClass(_pool.FindMessageTypeByName(f"{PACKAGE}.{_name}")))
for _ename, _vals in ENUMS.items():
    _ed = _pool.FindEnumTypeByName(f"{PACKAGE}.{_ename}")
    setattr(pb, _ename, _ed)
    for _vn, _num in _vals:
        setattr(pb, _vn if _ename != "DataType" else f"DT_{_vn}", _num)

# Convenience aliases
IN_PROGRESS, SUCCESS, FAILED = 0, 1, 2
SUM, PROD, MIN, MAX = 0, 1, 2, 3
DT_FLOAT32, DT_UINT8, DT_BFLOAT16, DT_FLOAT16, DT_INT32 = 0, 1, 2, 3, 4
DT_SIZE = {DT_FLOAT32: 4, DT_UINT8: 1, DT_BFLOAT16: 2, DT_FLOAT16: 2, DT_INT32: 4}


def method_path(service: str, method: str) -> str:
    return f"/{PACKAGE}.{service}/{method}"


def service_methods(service: str):
    for meth, req, resp, cstream in SERVICES[service]:
        yield meth, getattr(pb, req), getattr(pb, resp), cstream
