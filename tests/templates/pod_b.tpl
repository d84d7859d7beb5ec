{{ $ts := .metadata.creationTimestamp }}
conditions: [{type: Ready, status: "True", lastTransitionTime: "{{ $ts }}"}]
{{ if .spec.initContainers }}
initContainerStatuses:
{{- range .spec.initContainers }}
- name: {{ .name }}
  state: {terminated: {reason: Completed, exitCode: 0, finishedAt: "{{ $ts }}"}}
{{- end }}
{{ else }}
initContainerStatuses: []
{{ end }}
{{ with .status -}}
hostIP: "{{ with .hostIP }}{{ . }}{{ else }}{{ NodeIP }}{{ end }}"
podIP: '{{ with .podIP }}{{ . }}{{ else }}{{ PodIP }}{{ end }}'
{{- end }}
message: started at {{ StartTime }}  # a comment
phase: Running
startTime: {{ $ts }}
