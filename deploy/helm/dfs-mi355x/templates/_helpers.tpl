{{- define "dfs.name" -}}{{ .Release.Name }}-dfs{{- end -}}
{{- define "dfs.labels" -}}
app.kubernetes.io/name: dfs-mi355x
app.kubernetes.io/instance: {{ .Release.Name }}
{{- end -}}
{{- define "dfs.image" -}}{{ .Values.image.repository }}:{{ .Values.image.tag }}{{- end -}}
{{- define "dfs.configServers" -}}
{{- $n := int .Values.configserver.replicas -}}
{{- $root := . -}}
{{- range $i := until $n -}}{{ if $i }},{{ end }}http://{{ include "dfs.name" $root }}-config-{{ $i }}.{{ include "dfs.name" $root }}-config:{{ $root.Values.configserver.port }}{{- end -}}
{{- end -}}
