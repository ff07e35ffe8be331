{{- define "llmd.name" -}}{{ .Release.Name }}{{- end -}}
{{- define "llmd.pool" -}}{{ default (printf "%s-pool" .Release.Name) .Values.inferencePool.name }}{{- end -}}
{{- define "llmd.image" -}}{{ .Values.image.repository }}:{{ .Values.image.tag }}{{- end -}}
{{- define "llmd.served" -}}{{ default .Values.model.name .Values.model.servedName }}{{- end -}}
{{- define "llmd.labels" -}}
app.kubernetes.io/instance: {{ .Release.Name }}
app.kubernetes.io/part-of: llmd-amd
{{- end -}}
{{- define "llmd.engineArgs" -}}
- --model
- {{ .root.Values.model.name | quote }}
- --served-model-name
- {{ include "llmd.served" .root | quote }}
- --load-format
- {{ .root.Values.model.loadFormat }}
{{- if .root.Values.model.weights.pvc }}
- --weights-path
- {{ .root.Values.model.weights.mountPath }}
{{- end }}
- --tensor-parallel-size
- {{ .tp | quote }}
{{- if .root.Values.kvEvents.enabled }}
- --kv-events-config
- {{ printf "{\"enable_kv_cache_events\":true,\"publisher\":\"zmq\",\"endpoint\":\"tcp://*:%v\",\"topic\":\"kv@$(POD_IP):%v@%s\"}" .root.Values.kvEvents.port .port (include "llmd.served" .root) | quote }}
{{- end }}
{{- if .root.Values.kvOffload.enabled }}
- --kv-offload-config
- {{ printf "{\"cpu_bytes_to_use\":%v,\"fs_root\":\"%s\"}" (int64 .root.Values.kvOffload.cpuBytes) .root.Values.kvOffload.fsRoot | quote }}
{{- end }}
{{- end -}}
