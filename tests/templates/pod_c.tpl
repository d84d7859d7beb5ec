{{ $t := .metadata.creationTimestamp }}
conditions:
- lastTransitionTime: {{ $t }}
  status: "True"
  type: Ready
containerStatuses:
{{ range .spec.containers }}
- image: {{ .image }}
  name: {{ .name }}
  ready: true
  restartCount: 0
  state:
    running:
      startedAt: {{ $t }}
{{ end }}
ephemeral: none
{{ with .status }}
hostIP: {{ with .hostIP }}{{ . }}{{ else }}{{ NodeIP }}{{ end }}
podIP: {{ with .podIP }}{{ . }}{{ else }}{{ PodIP }}{{ end }}
{{ end }}
hostIPs: {{ $t }}
phase: Running
podIPs: {{ $t }}
qosClass: BestEffort
startTime: {{ $t }}
