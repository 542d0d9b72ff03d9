function radar_processing(process_animal_activity)
%RADAR_PROCESSING  MI355X drop-in for radar-etl-pipeline/radar_processing.m.
%   Same signature, inputs (radar_data.xml / radar_data.raw.bin in pwd via
%   f_parse_data2) and JSON outputs as the reference; the per-frame loop
%   (:197-261) and the STFT (:270-299) run in libfmcw through fmcw_mex.
%   Called unchanged by radar_processing_with_azure.m:50.  See INTEGRATION.md.
%
%   Host-side steps kept in MATLAB: parsing (:86), params (:89-154),
%   calibration (:166-174), the measurement update with its (fr_idx, j)
%   growth (:242-252) and the uploads; the JSON files and spectrogram.png are
%   written by libfmcw (fmcw_mex 'json' / 'stft_png').

addpath("lib");
fdata = 'radar_data';
[~, filename, ~] = fileparts(fdata);
if ~exist('xml2struct', 'file')
    error("Missing required function: xml2struct.m. Ensure it is included in the deployed files.");
end
[frame, frame_count, calib_data, sXML] = f_parse_data2(fdata);

% ---- parameters (reference :89-154) ------------------------------------------
dev = sXML.Device;
fmcw = dev.FmcwEndpoint.FmcwConfiguration;
up_khz = str2double(fmcw.upperFrequency_kHz.Text);
lo_khz = str2double(fmcw.lowerFrequency_kHz.Text);
prt = str2double(dev.BaseEndpoint.chirpDuration_ns.Text) * 1e-9 + 200e-6 + 300e-6;
bw = (up_khz - lo_khz) * 1e3;
fc = (up_khz + lo_khz) / 2 * 1e3;
n_rx = str2double(dev.BaseEndpoint.DeviceInfo.numAntennasRx.Text);
nts = str2double(dev.BaseEndpoint.FrameFormat.numSamplesPerChirp.Text);
pn = str2double(dev.BaseEndpoint.FrameFormat.numChirpsPerFrame.Text);
nr = 256; nd = 16;                       % literal FFT sizes of the reference
lambda = 3e8 / fc;
dist_per_bin = (nts * 3e8 / (2 * bw)) / nr;
fd_per_bin = (1 / (2 * prt)) / nd;

P = struct('nts', nts, 'pn', pn, 'nr', nr, 'nd', nd, 'max_targets', 1, ...
           'doppler_fallback_idx', 9, 'if_scale', 16 * 3.3 * nr / nts, ...
           'range_thr', 200, 'doppler_thr', 50, 'min_d', 0.9, 'max_d', 25.0, ...
           'dist_per_bin', dist_per_bin);

% ---- calibration + taps (reference :138-139, :166-174) -------------------------
n_cal = length(calib_data) / (2 * n_rx);
step = n_cal / nts;
cal = complex(calib_data(1:step:n_cal), calib_data(n_cal+1:step:2*n_cal)).';
fmcw_mex('init');                        % FMCW_DEVICES (e.g. '0,1,2,3'), else every visible GPU
used_devices = fmcw_mex('devices');
fprintf('radar_processing: DSP on %d GPU(s): %s\n', numel(used_devices), mat2str(used_devices));
fmcw_mex('taps', P, single(2 * blackman(nts)), single(2 * chebwin(pn)), single(complex(cal)));

% ---- the loop on the GPU (reference :197-261) ----------------------------------
iq = complex(zeros(nts, pn, frame_count, 'single'));
for f = 1:frame_count
    iq(:, :, f) = single(frame(f).Chirp(:, :, 1));
end
probe_col = 100;                         % reference :410
% range_tx1rx1_complete(:,100) needs pn*frame_count >= 100 (reference :411); the
% reference writes its first three JSON files before failing there, so the
% probe is only requested when it exists and the error is raised at :411 below
have_probe = pn * frame_count >= probe_col;
[prof, cnt, ridx, rmag, didx, slow, probe] = fmcw_mex('process', P, iq, probe_col * have_probe);
prof = double(prof); ridx = double(ridx); rmag = double(rmag); didx = double(didx);
to_speed = @(d) (d - nd/2 - 1) * -fd_per_bin * lambda / 2;

if strcmpi(process_animal_activity, 'no')
    % measurement update exactly as the reference writes it (:157-159, :242-252)
    meas.strength = zeros(1, frame_count); meas.range = zeros(1, frame_count); meas.speed = zeros(1, frame_count);
    for f = 1:frame_count
        for j = 1:cnt(f)
            meas.strength(f, j) = rmag(j, f);
            meas.range(f, j) = (ridx(j, f) - 1) * dist_per_bin;
            meas.speed(f, j) = to_speed(didx(j, f));
        end
    end
    iq_data = reshape(slow(:, cnt > 0), 1, []);          % :257-260, :270
    % :270-299 and the spectrogram.png of :331-348, both from the one device STFT
    [T, log_freq_bins, intensity] = fmcw_mex('stft_png', iq_data, single(kaiser(20, 3)), 19, 0, 1/prt, 1024, ...
                                             'spectrogram.png');
    spec = struct('time', double(T), 'frequency', double(log_freq_bins), 'intensity', double(intensity), ...
                  'title', 'All Frames - Log-Scaled Spectrogram', 'xLabel', 'Time (s)', 'yLabel', 'Frequency (Hz)');
    emit('spectrogram_data.json', spec);
    send_picture_to_blob_storage('spectrogram.png');     % :347

    t_axis = (0:frame_count-1) * 0.15;
    emit([filename, '_range_fft_data.json'], struct('time_axis', t_axis, ...
         'array_bin_range', (0:nr-1) * dist_per_bin, 'range_tx1rx1_max_abs', prof, 'filename', filename));
    emit([filename, '_range_speed_data.json'], struct('time_axis', t_axis, ...
         'range', meas.range, 'speed', meas.speed, 'filename', filename));
    if ~have_probe
        error('MATLAB:badsubscript', 'Index in position 2 exceeds array bounds (must not exceed %d).', pn * frame_count);
    end
    emit([filename, '_fft_data.json'], struct('range_bins', 0:nr-1, 'magnitude', double(probe), ...
         'frame_index', probe_col, 'filename', filename));

elseif strcmpi(process_animal_activity, 'yes')
    nbatch = ceil(frame_count / 100);
    made = 0;
    for b = 1:nbatch
        fr = (b-1)*100 + 1 : min(b*100, frame_count);
        sel = fr(cnt(fr) > 0);
        x = reshape(slow(:, sel), 1, []);
        if isempty(x) || numel(x) < 20
            continue;
        end
        made = made + 1;
        if made > 4
            break;
        end
        [T, fq, inten] = fmcw_mex('stft', x, single(kaiser(20, 3)), 19, 0, 1/prt, 1024);
        out = struct('time', double(T), 'frequency', double(fq), 'intensity', double(inten), ...
                     'title', ['Spectrogram - Batch ', num2str(b)], ...
                     'xLabel', 'Time (s) (relative to detected activity)', 'yLabel', 'Frequency (Hz)', ...
                     'start_frame', fr(1), 'end_frame', fr(end), 'filename_base', filename);
        emit([filename, '_spectrogram_batch_', num2str(b), '.json'], out);
    end
end
end

function emit(name, s)
% write one JSON file and upload it (reference :313-328 and friends): jsonencode(s,
% 'PrettyPrint', true) + fprintf, natively in libfmcw (fmcw_json_write)
try
    fmcw_mex('json', name, s);
catch err
    disp(['Error: Could not write ', name, ': ', err.message]);
    return;
end
send_json_string_to_blob_storage(name);
end
