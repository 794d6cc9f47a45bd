"""tfplugin5 protocol messages, built at import time from descriptors (no ``protoc`` here).

Field numbers follow Terraform's ``tfplugin5.2`` protocol, the one
``terraform-plugin-sdk/v2`` serves (reference ``main.go:13`` -> ``plugin.Serve``).
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

F = descriptor_pb2.FieldDescriptorProto
PKG = "tfplugin5"

# (name, number, type, label, type_name)
_T = {"string": F.TYPE_STRING, "bytes": F.TYPE_BYTES, "bool": F.TYPE_BOOL,
      "int64": F.TYPE_INT64, "enum": F.TYPE_ENUM, "msg": F.TYPE_MESSAGE}


def _field(msg, name, number, kind, repeated=False, type_name=None, oneof=None):
    f = msg.field.add()
    f.name = name
    f.number = number
    f.type = _T[kind]
    f.label = F.LABEL_REPEATED if repeated else F.LABEL_OPTIONAL
    if type_name:
        f.type_name = type_name if type_name.startswith(".") else "." + PKG + "." + type_name
    if oneof is not None:
        f.oneof_index = oneof
    return f


def _map_entry(parent, field_name, number, value_kind, value_type=None):
    entry_name = "".join(p.capitalize() for p in field_name.split("_")) + "Entry"
    entry = parent.nested_type.add()
    entry.name = entry_name
    entry.options.map_entry = True
    _field(entry, "key", 1, "string")
    _field(entry, "value", 2, value_kind, type_name=value_type)
    _field(parent, field_name, number, "msg", repeated=True,
           type_name=parent.name + "." + entry_name if "." not in parent.name else None)
    return entry


def _build() -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto()
    fd.name = "tfplugin5.proto"
    fd.package = PKG
    fd.syntax = "proto3"

    dv = fd.message_type.add(name="DynamicValue")
    _field(dv, "msgpack", 1, "bytes")
    _field(dv, "json", 2, "bytes")

    ap = fd.message_type.add(name="AttributePath")
    step = ap.nested_type.add(name="Step")
    step.oneof_decl.add(name="selector")
    _field(step, "attribute_name", 1, "string", oneof=0)
    _field(step, "element_key_string", 2, "string", oneof=0)
    _field(step, "element_key_int", 3, "int64", oneof=0)
    _field(ap, "steps", 1, "msg", repeated=True, type_name="AttributePath.Step")

    diag = fd.message_type.add(name="Diagnostic")
    sev = diag.enum_type.add(name="Severity")
    for i, n in enumerate(("INVALID", "ERROR", "WARNING")):
        sev.value.add(name=n, number=i)
    _field(diag, "severity", 1, "enum", type_name="Diagnostic.Severity")
    _field(diag, "summary", 2, "string")
    _field(diag, "detail", 3, "string")
    _field(diag, "attribute", 4, "msg", type_name="AttributePath")

    sk = fd.enum_type.add(name="StringKind")
    sk.value.add(name="PLAIN", number=0)
    sk.value.add(name="MARKDOWN", number=1)

    stop = fd.message_type.add(name="Stop")
    stop.nested_type.add(name="Request")
    r = stop.nested_type.add(name="Response")
    _field(r, "Error", 1, "string")

    raw = fd.message_type.add(name="RawState")
    _field(raw, "json", 1, "bytes")
    entry = raw.nested_type.add(name="FlatmapEntry")
    entry.options.map_entry = True
    _field(entry, "key", 1, "string")
    _field(entry, "value", 2, "string")
    _field(raw, "flatmap", 2, "msg", repeated=True, type_name="RawState.FlatmapEntry")

    schema = fd.message_type.add(name="Schema")
    block = schema.nested_type.add(name="Block")
    _field(block, "version", 1, "int64")
    _field(block, "attributes", 2, "msg", repeated=True, type_name="Schema.Attribute")
    _field(block, "block_types", 3, "msg", repeated=True, type_name="Schema.NestedBlock")
    _field(block, "description", 4, "string")
    _field(block, "description_kind", 5, "enum", type_name="StringKind")
    _field(block, "deprecated", 6, "bool")
    attr = schema.nested_type.add(name="Attribute")
    _field(attr, "name", 1, "string")
    _field(attr, "type", 2, "bytes")
    _field(attr, "description", 3, "string")
    _field(attr, "required", 4, "bool")
    _field(attr, "optional", 5, "bool")
    _field(attr, "computed", 6, "bool")
    _field(attr, "sensitive", 7, "bool")
    _field(attr, "description_kind", 8, "enum", type_name="StringKind")
    _field(attr, "deprecated", 9, "bool")
    nb = schema.nested_type.add(name="NestedBlock")
    nm = nb.enum_type.add(name="NestingMode")
    for i, n in enumerate(("INVALID", "SINGLE", "LIST", "SET", "MAP", "GROUP")):
        nm.value.add(name=n, number=i)
    _field(nb, "type_name", 1, "string")
    _field(nb, "block", 2, "msg", type_name="Schema.Block")
    _field(nb, "nesting", 3, "enum", type_name="Schema.NestedBlock.NestingMode")
    _field(nb, "min_items", 4, "int64")
    _field(nb, "max_items", 5, "int64")
    _field(schema, "version", 1, "int64")
    _field(schema, "block", 2, "msg", type_name="Schema.Block")

    gps = fd.message_type.add(name="GetProviderSchema")
    gps.nested_type.add(name="Request")
    caps = gps.nested_type.add(name="ServerCapabilities")
    _field(caps, "plan_destroy", 1, "bool")
    resp = gps.nested_type.add(name="Response")
    _field(resp, "provider", 1, "msg", type_name="Schema")
    for fname, num in (("resource_schemas", 2), ("data_source_schemas", 3)):
        e = resp.nested_type.add(name="".join(p.capitalize() for p in fname.split("_")) + "Entry")
        e.options.map_entry = True
        _field(e, "key", 1, "string")
        _field(e, "value", 2, "msg", type_name="Schema")
        _field(resp, fname, num, "msg", repeated=True,
               type_name="GetProviderSchema.Response." + e.name)
    _field(resp, "diagnostics", 4, "msg", repeated=True, type_name="Diagnostic")
    _field(resp, "provider_meta", 5, "msg", type_name="Schema")
    _field(resp, "server_capabilities", 6, "msg", type_name="GetProviderSchema.ServerCapabilities")

    def rpc_msg(name, request, response):
        m = fd.message_type.add(name=name)
        req = m.nested_type.add(name="Request")
        for spec in request:
            _field(req, *spec)
        res = m.nested_type.add(name="Response")
        for spec in response:
            _field(res, *spec)
        return m

    diags = lambda n: ("diagnostics", n, "msg", True, "Diagnostic")  # noqa: E731
    rpc_msg("PrepareProviderConfig", [("config", 1, "msg", False, "DynamicValue")],
            [("prepared_config", 1, "msg", False, "DynamicValue"), diags(2)])
    rpc_msg("UpgradeResourceState", [("type_name", 1, "string"), ("version", 2, "int64"),
                                     ("raw_state", 3, "msg", False, "RawState")],
            [("upgraded_state", 1, "msg", False, "DynamicValue"), diags(2)])
    rpc_msg("ValidateResourceTypeConfig", [("type_name", 1, "string"),
                                           ("config", 2, "msg", False, "DynamicValue")],
            [diags(1)])
    rpc_msg("ValidateDataSourceConfig", [("type_name", 1, "string"),
                                         ("config", 2, "msg", False, "DynamicValue")], [diags(1)])
    rpc_msg("Configure", [("terraform_version", 1, "string"),
                          ("config", 2, "msg", False, "DynamicValue")], [diags(1)])
    rpc_msg("ReadResource", [("type_name", 1, "string"),
                             ("current_state", 2, "msg", False, "DynamicValue"),
                             ("private", 3, "bytes"),
                             ("provider_meta", 4, "msg", False, "DynamicValue")],
            [("new_state", 1, "msg", False, "DynamicValue"), diags(2), ("private", 3, "bytes")])
    rpc_msg("PlanResourceChange", [("type_name", 1, "string"),
                                   ("prior_state", 2, "msg", False, "DynamicValue"),
                                   ("proposed_new_state", 3, "msg", False, "DynamicValue"),
                                   ("config", 4, "msg", False, "DynamicValue"),
                                   ("prior_private", 5, "bytes"),
                                   ("provider_meta", 6, "msg", False, "DynamicValue")],
            [("planned_state", 1, "msg", False, "DynamicValue"),
             ("requires_replace", 2, "msg", True, "AttributePath"),
             ("planned_private", 3, "bytes"), diags(4), ("legacy_type_system", 5, "bool")])
    rpc_msg("ApplyResourceChange", [("type_name", 1, "string"),
                                    ("prior_state", 2, "msg", False, "DynamicValue"),
                                    ("planned_state", 3, "msg", False, "DynamicValue"),
                                    ("config", 4, "msg", False, "DynamicValue"),
                                    ("planned_private", 5, "bytes"),
                                    ("provider_meta", 6, "msg", False, "DynamicValue")],
            [("new_state", 1, "msg", False, "DynamicValue"), ("private", 2, "bytes"), diags(3),
             ("legacy_type_system", 4, "bool")])
    imp = rpc_msg("ImportResourceState", [("type_name", 1, "string"), ("id", 2, "string")], [])
    ir = imp.nested_type.add(name="ImportedResource")
    _field(ir, "type_name", 1, "string")
    _field(ir, "state", 2, "msg", type_name="DynamicValue")
    _field(ir, "private", 3, "bytes")
    ires = [m for m in imp.nested_type if m.name == "Response"][0]
    _field(ires, "imported_resources", 1, "msg", True, "ImportResourceState.ImportedResource")
    _field(ires, "diagnostics", 2, "msg", True, "Diagnostic")
    rpc_msg("ReadDataSource", [("type_name", 1, "string"),
                               ("config", 2, "msg", False, "DynamicValue"),
                               ("provider_meta", 3, "msg", False, "DynamicValue")],
            [("state", 1, "msg", False, "DynamicValue"), diags(2)])
    return fd


_pool = descriptor_pool.DescriptorPool()
_file = _pool.Add(_build())


def message(name: str):
    return message_factory.GetMessageClass(_pool.FindMessageTypeByName(PKG + "." + name))


DynamicValue = message("DynamicValue")
AttributePath = message("AttributePath")
Diagnostic = message("Diagnostic")
Schema = message("Schema")

# service method -> (request class, response class)
METHODS = {
    "GetSchema": ("GetProviderSchema.Request", "GetProviderSchema.Response"),
    "PrepareProviderConfig": ("PrepareProviderConfig.Request", "PrepareProviderConfig.Response"),
    "ValidateResourceTypeConfig": ("ValidateResourceTypeConfig.Request",
                                   "ValidateResourceTypeConfig.Response"),
    "ValidateDataSourceConfig": ("ValidateDataSourceConfig.Request",
                                 "ValidateDataSourceConfig.Response"),
    "UpgradeResourceState": ("UpgradeResourceState.Request", "UpgradeResourceState.Response"),
    "Configure": ("Configure.Request", "Configure.Response"),
    "ReadResource": ("ReadResource.Request", "ReadResource.Response"),
    "PlanResourceChange": ("PlanResourceChange.Request", "PlanResourceChange.Response"),
    "ApplyResourceChange": ("ApplyResourceChange.Request", "ApplyResourceChange.Response"),
    "ImportResourceState": ("ImportResourceState.Request", "ImportResourceState.Response"),
    "ReadDataSource": ("ReadDataSource.Request", "ReadDataSource.Response"),
    "Stop": ("Stop.Request", "Stop.Response"),
}
SERVICE = "tfplugin5.Provider"


def classes(method: str):
    req, res = METHODS[method]
    return message(req), message(res)
