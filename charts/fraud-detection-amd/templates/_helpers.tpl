{{- define "fdx.name" -}}{{ .Release.Name }}{{- end -}}
{{- define "fdx.image" -}}{{ .Values.image.repository }}:{{ .Values.image.tag }}{{- end -}}
{{- define "fdx.labels" -}}
app.kubernetes.io/name: fraud-detection-amd
app.kubernetes.io/instance: {{ .Release.Name }}
app.kubernetes.io/version: {{ .Chart.AppVersion | quote }}
{{- end -}}
{{- define "fdx.envFrom" -}}
- configMapRef: {name: {{ include "fdx.name" . }}-config}
- secretRef: {name: {{ include "fdx.name" . }}-db}
{{- end -}}
{{- define "fdx.pullSecrets" -}}
{{- range .Values.imagePullSecrets }}
- name: {{ . }}
{{- end }}
{{- end -}}
