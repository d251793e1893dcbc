"""OTLP protobuf message classes built at run time from descriptor_pb2 (no
protoc and no opentelemetry-proto package in this image).

Restates the subset of opentelemetry-proto v1 the spanmetrics path reads and
writes (common/v1 AnyValue/KeyValue/InstrumentationScope, resource/v1 Resource,
trace/v1 Span..., metrics/v1 Sum/Histogram/Gauge...).  Field numbers and types
follow the published .proto files; only the wire format matters for the tests,
which use these classes as an independent protobuf implementation to check the
Node host's hand-written codec (host/node/lib/otlp.js) in both directions.
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

F = descriptor_pb2.FieldDescriptorProto
OPT, REP = F.LABEL_OPTIONAL, F.LABEL_REPEATED

# (name, number, type, label, type_name or None, oneof index or None, proto3_optional)
_MESSAGES = {
    "AnyValue": [
        ("string_value", 1, F.TYPE_STRING, OPT, None, 0),
        ("bool_value", 2, F.TYPE_BOOL, OPT, None, 0),
        ("int_value", 3, F.TYPE_INT64, OPT, None, 0),
        ("double_value", 4, F.TYPE_DOUBLE, OPT, None, 0),
        ("array_value", 5, F.TYPE_MESSAGE, OPT, "ArrayValue", 0),
        ("kvlist_value", 6, F.TYPE_MESSAGE, OPT, "KeyValueList", 0),
        ("bytes_value", 7, F.TYPE_BYTES, OPT, None, 0),
    ],
    "ArrayValue": [("values", 1, F.TYPE_MESSAGE, REP, "AnyValue", None)],
    "KeyValueList": [("values", 1, F.TYPE_MESSAGE, REP, "KeyValue", None)],
    "KeyValue": [("key", 1, F.TYPE_STRING, OPT, None, None),
                 ("value", 2, F.TYPE_MESSAGE, OPT, "AnyValue", None)],
    "InstrumentationScope": [("name", 1, F.TYPE_STRING, OPT, None, None),
                             ("version", 2, F.TYPE_STRING, OPT, None, None),
                             ("attributes", 3, F.TYPE_MESSAGE, REP, "KeyValue", None),
                             ("dropped_attributes_count", 4, F.TYPE_UINT32, OPT, None, None)],
    "Resource": [("attributes", 1, F.TYPE_MESSAGE, REP, "KeyValue", None),
                 ("dropped_attributes_count", 2, F.TYPE_UINT32, OPT, None, None)],
    "Status": [("message", 2, F.TYPE_STRING, OPT, None, None),
               ("code", 3, F.TYPE_INT32, OPT, None, None)],
    "Event": [("time_unix_nano", 1, F.TYPE_FIXED64, OPT, None, None),
              ("name", 2, F.TYPE_STRING, OPT, None, None),
              ("attributes", 3, F.TYPE_MESSAGE, REP, "KeyValue", None)],
    "Span": [("trace_id", 1, F.TYPE_BYTES, OPT, None, None),
             ("span_id", 2, F.TYPE_BYTES, OPT, None, None),
             ("trace_state", 3, F.TYPE_STRING, OPT, None, None),
             ("parent_span_id", 4, F.TYPE_BYTES, OPT, None, None),
             ("name", 5, F.TYPE_STRING, OPT, None, None),
             ("kind", 6, F.TYPE_INT32, OPT, None, None),
             ("start_time_unix_nano", 7, F.TYPE_FIXED64, OPT, None, None),
             ("end_time_unix_nano", 8, F.TYPE_FIXED64, OPT, None, None),
             ("attributes", 9, F.TYPE_MESSAGE, REP, "KeyValue", None),
             ("dropped_attributes_count", 10, F.TYPE_UINT32, OPT, None, None),
             ("events", 11, F.TYPE_MESSAGE, REP, "Event", None),
             ("status", 15, F.TYPE_MESSAGE, OPT, "Status", None),
             ("flags", 16, F.TYPE_FIXED32, OPT, None, None)],
    "ScopeSpans": [("scope", 1, F.TYPE_MESSAGE, OPT, "InstrumentationScope", None),
                   ("spans", 2, F.TYPE_MESSAGE, REP, "Span", None),
                   ("schema_url", 3, F.TYPE_STRING, OPT, None, None)],
    "ResourceSpans": [("resource", 1, F.TYPE_MESSAGE, OPT, "Resource", None),
                      ("scope_spans", 2, F.TYPE_MESSAGE, REP, "ScopeSpans", None),
                      ("schema_url", 3, F.TYPE_STRING, OPT, None, None)],
    "ExportTraceServiceRequest": [("resource_spans", 1, F.TYPE_MESSAGE, REP, "ResourceSpans", None)],
    "NumberDataPoint": [("attributes", 7, F.TYPE_MESSAGE, REP, "KeyValue", None),
                        ("start_time_unix_nano", 2, F.TYPE_FIXED64, OPT, None, None),
                        ("time_unix_nano", 3, F.TYPE_FIXED64, OPT, None, None),
                        ("as_double", 4, F.TYPE_DOUBLE, OPT, None, 0),
                        ("as_int", 6, F.TYPE_SFIXED64, OPT, None, 0),
                        ("flags", 8, F.TYPE_UINT32, OPT, None, None)],
    "HistogramDataPoint": [("attributes", 9, F.TYPE_MESSAGE, REP, "KeyValue", None),
                           ("start_time_unix_nano", 2, F.TYPE_FIXED64, OPT, None, None),
                           ("time_unix_nano", 3, F.TYPE_FIXED64, OPT, None, None),
                           ("count", 4, F.TYPE_FIXED64, OPT, None, None),
                           ("sum", 5, F.TYPE_DOUBLE, OPT, None, "proto3_optional"),
                           ("bucket_counts", 6, F.TYPE_FIXED64, REP, None, None),
                           ("explicit_bounds", 7, F.TYPE_DOUBLE, REP, None, None),
                           ("flags", 10, F.TYPE_UINT32, OPT, None, None)],
    "Gauge": [("data_points", 1, F.TYPE_MESSAGE, REP, "NumberDataPoint", None)],
    "Sum": [("data_points", 1, F.TYPE_MESSAGE, REP, "NumberDataPoint", None),
            ("aggregation_temporality", 2, F.TYPE_INT32, OPT, None, None),
            ("is_monotonic", 3, F.TYPE_BOOL, OPT, None, None)],
    "Histogram": [("data_points", 1, F.TYPE_MESSAGE, REP, "HistogramDataPoint", None),
                  ("aggregation_temporality", 2, F.TYPE_INT32, OPT, None, None)],
    # ExponentialHistogramDataPoint.Buckets (nested upstream; the name is not on the wire)
    "ExpoBuckets": [("offset", 1, F.TYPE_SINT32, OPT, None, None),
                    ("bucket_counts", 2, F.TYPE_UINT64, REP, None, None)],
    "ExponentialHistogramDataPoint": [("attributes", 1, F.TYPE_MESSAGE, REP, "KeyValue", None),
                                      ("start_time_unix_nano", 2, F.TYPE_FIXED64, OPT, None, None),
                                      ("time_unix_nano", 3, F.TYPE_FIXED64, OPT, None, None),
                                      ("count", 4, F.TYPE_FIXED64, OPT, None, None),
                                      ("sum", 5, F.TYPE_DOUBLE, OPT, None, "proto3_optional"),
                                      ("scale", 6, F.TYPE_SINT32, OPT, None, None),
                                      ("zero_count", 7, F.TYPE_FIXED64, OPT, None, None),
                                      ("positive", 8, F.TYPE_MESSAGE, OPT, "ExpoBuckets", None),
                                      ("negative", 9, F.TYPE_MESSAGE, OPT, "ExpoBuckets", None),
                                      ("flags", 10, F.TYPE_UINT32, OPT, None, None),
                                      ("min", 12, F.TYPE_DOUBLE, OPT, None, "proto3_optional"),
                                      ("max", 13, F.TYPE_DOUBLE, OPT, None, "proto3_optional"),
                                      ("zero_threshold", 14, F.TYPE_DOUBLE, OPT, None, None)],
    "ExponentialHistogram": [("data_points", 1, F.TYPE_MESSAGE, REP, "ExponentialHistogramDataPoint", None),
                             ("aggregation_temporality", 2, F.TYPE_INT32, OPT, None, None)],
    "Metric": [("name", 1, F.TYPE_STRING, OPT, None, None),
               ("description", 2, F.TYPE_STRING, OPT, None, None),
               ("unit", 3, F.TYPE_STRING, OPT, None, None),
               ("gauge", 5, F.TYPE_MESSAGE, OPT, "Gauge", 0),
               ("sum", 7, F.TYPE_MESSAGE, OPT, "Sum", 0),
               ("histogram", 9, F.TYPE_MESSAGE, OPT, "Histogram", 0),
               ("exponential_histogram", 10, F.TYPE_MESSAGE, OPT, "ExponentialHistogram", 0)],
    "ScopeMetrics": [("scope", 1, F.TYPE_MESSAGE, OPT, "InstrumentationScope", None),
                     ("metrics", 2, F.TYPE_MESSAGE, REP, "Metric", None),
                     ("schema_url", 3, F.TYPE_STRING, OPT, None, None)],
    "ResourceMetrics": [("resource", 1, F.TYPE_MESSAGE, OPT, "Resource", None),
                        ("scope_metrics", 2, F.TYPE_MESSAGE, REP, "ScopeMetrics", None),
                        ("schema_url", 3, F.TYPE_STRING, OPT, None, None)],
    "ExportMetricsServiceRequest": [("resource_metrics", 1, F.TYPE_MESSAGE, REP, "ResourceMetrics", None)],
}
_ONEOF_NAME = {"AnyValue": "value", "NumberDataPoint": "value", "Metric": "data"}
_PKG = "otlptest"


def _build():
    fd = descriptor_pb2.FileDescriptorProto(name="otlp_test.proto", package=_PKG, syntax="proto3")
    for msg, fields in _MESSAGES.items():
        m = fd.message_type.add(name=msg)
        if msg in _ONEOF_NAME:
            m.oneof_decl.add(name=_ONEOF_NAME[msg])
        for name, num, typ, label, tname, oneof in fields:
            f = m.field.add(name=name, number=num, type=typ, label=label)
            if tname:
                f.type_name = f".{_PKG}.{tname}"
            if oneof == "proto3_optional":
                # proto3 `optional` = a synthetic one-field oneof
                f.proto3_optional = True
                f.oneof_index = len(m.oneof_decl)
                m.oneof_decl.add(name="_" + name)
            elif oneof is not None:
                f.oneof_index = oneof
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    return {msg: message_factory.GetMessageClass(pool.FindMessageTypeByName(f"{_PKG}.{msg}"))
            for msg in _MESSAGES}


M = _build()
